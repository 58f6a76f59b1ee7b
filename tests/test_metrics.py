"""Metrics sources + manager rules against the FakeCluster (manager.go:493-565, sources/*.go)."""
import datetime as dt

import pytest

from k8s_llm_monitor_amd.monitor.cluster.backend import milli_value, parse_quantity, value, match_labels, match_fields
from k8s_llm_monitor_amd.monitor.cluster.fake import FakeCluster
from k8s_llm_monitor_amd.monitor.metrics.manager import ManagerConfig, MetricsManager, calculate_cluster_metrics
from k8s_llm_monitor_amd.monitor.metrics.sources import build_node_metrics, build_pod_metrics
from k8s_llm_monitor_amd.monitor.types import ClusterMetrics, MetricsSnapshot, NetworkMetrics, NodeMetrics, PodMetrics, UAVReport
from k8s_llm_monitor_amd.utils.gojson import utcnow


def test_quantities():
    assert milli_value("250m") == 250 and milli_value("2") == 2000 and milli_value("1500000n") == 2
    assert value("1Ki") == 1024 and value("1Gi") == 1 << 30 and value("128Mi") == 128 << 20 and value("1e3") == 1000
    assert parse_quantity("0.5") == 0.5


def test_selectors():
    assert match_labels("app=uav-agent", {"app": "uav-agent"})
    assert not match_labels("app=uav-agent,tier!=x", {"app": "uav-agent", "tier": "x"})
    assert match_labels("env in (a, b),!legacy", {"env": "b"})
    assert match_fields("status.phase=Running,spec.nodeName=n1", {"status": {"phase": "Running"}, "spec": {"nodeName": "n1"}})
    assert not match_fields("status.phase!=Running", {"status": {"phase": "Running"}})


@pytest.fixture()
def fc():
    return FakeCluster.build(seed=3)


def _mgr(fc, **kw):
    return MetricsManager(fc, ManagerConfig(namespaces=["default", "kube-system"], **kw))


def test_collect_snapshot(fc):
    m = _mgr(fc)
    s = m.collect()
    assert len(s.node_metrics) == 3 and all(n.healthy for n in s.node_metrics.values())
    assert s.cluster_metrics.total_pods == len(s.pod_metrics) > 5
    assert s.cluster_metrics.health_status == "healthy"
    n = next(iter(s.node_metrics.values()))
    assert n.cpu_capacity > 0 and 0 < n.cpu_usage_rate < 100 and n.gpu_models == [] and n.conditions is None
    uav = m.get_uav_metrics()
    assert len(uav) == 3 and all(e["source"] == "pull" and e["state"].battery.remaining_percent > 50 for e in uav.values())


def test_node_health_rules(fc):
    node = "k3d-k8s-llm-monitor-agent-0"
    fc.set_node_pressure(node, "MemoryPressure")
    s = _mgr(fc).collect()
    nm = s.node_metrics[node]
    assert not nm.healthy and nm.conditions[0].startswith("MemoryPressure:")
    assert s.cluster_metrics.issues[0] == "1 nodes are unhealthy"
    fc.set_node_ready(node, False)
    s = _mgr(fc).collect()
    assert any(c.startswith("NotReady:") for c in s.node_metrics[node].conditions)
    assert s.node_metrics[node].cpu_usage == 0  # metrics-server cannot scrape a NotReady node


def test_metrics_server_down_degrades_to_zero(fc):
    fc.faults["metrics_down"] = True
    s = _mgr(fc).collect()
    assert all(n.cpu_usage == 0 for n in s.node_metrics.values())
    assert all(p.containers is None for p in s.pod_metrics.values())


def test_pod_metrics_rates_relative_to_limit(fc):
    fc.overload_pod("default", "redis-0", 0.95)
    s = _mgr(fc).collect()
    p = s.pod_metrics["default/redis-0"]
    assert p.memory_limit == 512 << 20 and p.memory_usage_rate > 90 and p.is_over_limit()
    assert p.cpu_usage_rate > 0 and p.containers[0].memory_limit == 512 << 20


def test_cluster_status_thresholds():
    def snap(nodes):
        return MetricsSnapshot(node_metrics=nodes, pod_metrics={}, network_metrics=[], cluster_metrics=ClusterMetrics())
    s = snap({"a": NodeMetrics(cpu_capacity=1000, cpu_usage=850, memory_capacity=100, memory_usage=10, healthy=True)})
    calculate_cluster_metrics(s)
    assert s.cluster_metrics.health_status == "warning" and s.cluster_metrics.issues == ["High CPU usage: 85.0%"]
    s = snap({"a": NodeMetrics(cpu_capacity=1000, cpu_usage=950, memory_capacity=100, memory_usage=10, healthy=True)})
    calculate_cluster_metrics(s)
    assert s.cluster_metrics.health_status == "critical"
    nodes = {str(i): NodeMetrics(cpu_capacity=10, memory_capacity=10, healthy=i < 1) for i in range(4)}
    s = snap(nodes)
    calculate_cluster_metrics(s)
    assert s.cluster_metrics.health_status == "critical" and s.cluster_metrics.issues == ["3 nodes are unhealthy"]
    nodes = {"g": NodeMetrics(gpu_count=2, gpu_usage=[10.0, 70.0], healthy=True)}
    s = snap(nodes)
    calculate_cluster_metrics(s)
    assert (s.cluster_metrics.total_gpus, s.cluster_metrics.available_gpus) == (2, 1)


def test_helpers():
    assert NodeMetrics(disk_usage_rate=91).is_under_pressure()
    assert not NodeMetrics(cpu_usage_rate=80).is_under_pressure()
    p = PodMetrics(cpu_usage=90, cpu_limit=100, cpu_request=50, memory_usage=10, memory_request=20)
    assert p.is_over_limit() and p.get_resource_utilization() == (180.0, 50.0)
    assert NetworkMetrics(connected=True, rtt=9.9).get_quality() == "excellent"
    assert NetworkMetrics(connected=True, rtt=60).get_quality() == "fair"
    assert NetworkMetrics().get_quality() == "disconnected"


def test_uav_push_and_staleness(fc):
    m = _mgr(fc, enable_uav=False)
    old = utcnow() - dt.timedelta(seconds=100)
    m.update_uav_report(UAVReport(node_name="n1", uav_id="U1", timestamp=old, heartbeat_interval_seconds=10))
    m.update_uav_report(UAVReport(node_name="n2", uav_id="U2", heartbeat_interval_seconds=10))
    u = m.get_uav_metrics()
    assert u["n1"]["status"] == "stale" and u["n2"]["status"] == "active" and u["n2"]["source"] == "agent"
    assert m.get_single_uav_metrics("nope") is None


def test_pull_does_not_wipe_push_when_empty(fc):
    fc.faults["agent_down"] = {n for n in ["k3d-k8s-llm-monitor-server-0", "k3d-k8s-llm-monitor-agent-0",
                                           "k3d-k8s-llm-monitor-agent-1"]}
    m = _mgr(fc)
    m.update_uav_report(UAVReport(node_name="edge", uav_id="U"))
    m.collect()
    assert "edge" in m.get_uav_metrics()


def test_network_source_semaphore_and_pairs(fc):
    from k8s_llm_monitor_amd.monitor.analysis.network import RTTTester
    from k8s_llm_monitor_amd.monitor.cluster.client import K8sClient

    m = MetricsManager(fc, ManagerConfig(namespaces=["default"], enable_network=True, network_max_pairs=5),
                       RTTTester(K8sClient(fc)))
    s = m.collect()
    assert len(s.network_metrics) == 5
    assert all(x.source_pod.startswith("default/") for x in s.network_metrics)
    nodes = {p["metadata"]["name"]: p["spec"]["nodeName"] for p in fc.list(__import__("k8s_llm_monitor_amd.monitor.cluster.backend", fromlist=["PODS"]).PODS)}
    for x in s.network_metrics:  # cross-node pairs preferred
        assert nodes[x.source_pod.split("/")[1]] != nodes[x.target_pod.split("/")[1]]
