"""The stdlib Kubernetes REST client against a FakeCluster served on the real API paths."""
import threading
import time

import pytest

from k8s_llm_monitor_amd.monitor.cluster.backend import NODE_METRICS, NODES, PODS, UAV_METRICS, ApiError
from k8s_llm_monitor_amd.monitor.cluster.client import K8sClient
from k8s_llm_monitor_amd.monitor.cluster.fake import FakeCluster
from k8s_llm_monitor_amd.monitor.cluster.fake_apiserver import serve
from k8s_llm_monitor_amd.monitor.cluster.kube import KubeRESTBackend
from k8s_llm_monitor_amd.monitor.metrics.manager import ManagerConfig, MetricsManager
from k8s_llm_monitor_amd.monitor.types import UAVReport


@pytest.fixture()
def api():
    fc = FakeCluster.build(seed=4)
    srv = serve(fc, token="t0k")
    kb = KubeRESTBackend(f"http://127.0.0.1:{srv.server_address[1]}", token="t0k")
    yield fc, kb
    srv.shutdown()


def test_crud_and_selectors(api):
    fc, kb = api
    assert kb.server_version()["gitVersion"].startswith("v1.31")
    assert len(kb.list(NODES)) == 3
    agents = kb.list(PODS, "default", label_selector="app=uav-agent", field_selector="status.phase=Running")
    assert len(agents) == 3 and all(p["kind"] == "Pod" for p in agents)
    assert kb.get(PODS, "redis-0", "default")["metadata"]["name"] == "redis-0"
    with pytest.raises(ApiError) as e:
        kb.get(PODS, "nope", "default")
    assert e.value.not_found
    assert len(kb.list(NODE_METRICS)) == 3
    c = K8sClient(kb)
    assert c.upsert_uav_metric(UAVReport(node_name="n1", uav_id="U1")) == "created"
    assert c.upsert_uav_metric(UAVReport(node_name="n1", uav_id="U1", status="degraded")) == "updated"
    assert fc.get(UAV_METRICS, "uavmetric-n1", "default")["status"]["collection_status"] == "degraded"
    assert "started" in kb.pod_logs("default", "redis-0", 10)


def test_unauthorized():
    fc = FakeCluster.build(seed=4)
    srv = serve(fc, token="secret")
    try:
        with pytest.raises(ApiError) as e:
            KubeRESTBackend(f"http://127.0.0.1:{srv.server_address[1]}", token="wrong").list(NODES)
        assert e.value.code == 401
    finally:
        srv.shutdown()


def test_watch_stream(api):
    fc, kb = api
    got = []
    stop = threading.Event()

    def run():
        for etype, obj in kb.watch(PODS, "default", timeout_s=3, stop=stop):
            got.append((etype, obj["metadata"]["name"]))
            if etype == "MODIFIED":
                stop.set()
                return

    t = threading.Thread(target=run)
    t.start()
    time.sleep(0.5)
    fc.crashloop_pod("default", "redis-0")
    t.join(5)
    assert ("MODIFIED", "redis-0") in got and sum(1 for e, _ in got if e == "ADDED") >= 5


def test_manager_over_rest(api):
    fc, kb = api
    m = MetricsManager(kb, ManagerConfig(namespaces=["default", "kube-system"], enable_uav=False))
    s = m.collect()
    assert len(s.node_metrics) == 3 and s.cluster_metrics.total_pods > 5
