"""Rule-based analyzer + RTT tester (network.go, rtt_tester.go) incl. fault scenarios."""
import pytest

from k8s_llm_monitor_amd.monitor.analysis.network import (NetworkAnalyzer, RTTTester, assess_latency, is_http_service,
                                                          parse_http_output, parse_ping_output, parse_pod_name)
from k8s_llm_monitor_amd.monitor.cluster.client import K8sClient
from k8s_llm_monitor_amd.monitor.cluster.fake import FakeCluster
from k8s_llm_monitor_amd.monitor.types import ContainerInfo, PodInfo, RTTResult

IPUTILS = """PING 10.42.1.5 (10.42.1.5) 56(84) bytes of data.
64 bytes from 10.42.1.5: icmp_seq=1 ttl=62 time=0.412 ms
64 bytes from 10.42.1.5: icmp_seq=2 ttl=62 time=0.388 ms
64 bytes from 10.42.1.5: icmp_seq=3 ttl=62 time=0.401 ms

--- 10.42.1.5 ping statistics ---
3 packets transmitted, 3 received, 0% packet loss, time 2003ms
rtt min/avg/max/mdev = 0.388/0.400/0.412/0.009 ms
"""
BUSYBOX_LOSS = """PING 10.42.2.9 (10.42.2.9): 56 data bytes
64 bytes from 10.42.2.9: seq=0 ttl=62 time=1.250 ms

--- 10.42.2.9 ping statistics ---
3 packets transmitted, 1 packets received, 66% packet loss
"""


def test_ping_parsing():
    r = RTTResult()
    parse_ping_output(IPUTILS, r)
    assert r.success and abs(r.rtt - 0.4003333) < 1e-6 and r.packet_loss == 0
    r = RTTResult()
    parse_ping_output(BUSYBOX_LOSS, r)
    assert r.success and r.rtt == 1.25 and r.packet_loss == 66
    r = RTTResult()
    parse_ping_output("3 packets transmitted, 0 received, 100% packet loss", r)
    assert not r.success and r.packet_loss == 100


def test_http_parsing_and_grades():
    r = RTTResult()
    parse_http_output("0.002345\n", r)
    assert r.success and abs(r.rtt - 2.345) < 1e-9
    r = RTTResult()
    parse_http_output("", r)
    assert not r.success
    assert [assess_latency(x) for x in (0, 0.5, 3, 20, 70, 200)] == ["unknown", "excellent", "good", "fair", "poor",
                                                                      "very_poor"]


def test_helpers():
    assert parse_pod_name("kube-system/coredns") == ("kube-system", "coredns")
    assert parse_pod_name("web") == ("default", "web")
    assert is_http_service(PodInfo(labels={"app": "my-WEB-ui"}))
    assert is_http_service(PodInfo(containers=[ContainerInfo(image="docker.io/library/nginx:1.25")]))
    assert not is_http_service(PodInfo(labels={"app": "redis"}))


@pytest.fixture()
def fc():
    return FakeCluster.build(seed=5)


def test_healthy_pair_connected(fc):
    an = NetworkAnalyzer(K8sClient(fc))
    r = an.analyze_pod_communication("default/frontend-5c7d8f9b4-kq2lp", "default/nginx-web-6d4cf56db6-8v2mz")
    assert r.status == "connected" and r.confidence == 0.9 and r.issues == []
    assert r.solutions == ["No obvious issues detected"]
    methods = [x.method for x in an.last_rtt.rtt_results]
    assert methods == ["ping", "ping_reverse", "http"] and an.last_rtt.success_rate == 100
    assert an.last_rtt.latency == "excellent"


def test_rule_table(fc):
    c = K8sClient(fc)
    fc.fail_pod("default", "backend-84d6b7c5f-wx7rt")
    fc.set_coredns(False)
    r = NetworkAnalyzer(c, enable_rtt=False).analyze_pod_communication("default/frontend-5c7d8f9b4-kq2lp",
                                                                       "default/backend-84d6b7c5f-wx7rt")
    assert r.status == "disconnected" and r.confidence == 0.7
    assert "Pod default/backend-84d6b7c5f-wx7rt is not running (status: Failed)" in r.issues
    assert "CoreDNS is not running properly" in r.issues
    # redis has a NetworkPolicy selecting it; busybox has no Service
    r = NetworkAnalyzer(c, enable_rtt=False).analyze_pod_communication("default/redis-0", "default/busybox-test")
    assert "Network policy default/redis-allow-backend may affect communication" in r.issues
    assert "No service found targeting Pod default/busybox-test" in r.issues


def test_partition_and_latency_faults(fc):
    c = K8sClient(fc)
    fc.partition("k3d-k8s-llm-monitor-server-0", "k3d-k8s-llm-monitor-agent-0")
    r = NetworkAnalyzer(c).analyze_pod_communication("default/frontend-5c7d8f9b4-kq2lp", "default/nginx-web-6d4cf56db6-8v2mz")
    assert any("网络连通性差" in i for i in r.issues)
    fc.partition("k3d-k8s-llm-monitor-server-0", "k3d-k8s-llm-monitor-agent-0", on=False)
    fc.faults["extra_latency_ms"] = 60.0
    t = RTTTester(c).test_pod_connectivity("default/frontend-5c7d8f9b4-kq2lp", "default/nginx-web-6d4cf56db6-8v2mz")
    assert t.latency in ("poor", "very_poor")


def test_missing_pod_errors(fc):
    with pytest.raises(RuntimeError, match="failed to get pod A info"):
        NetworkAnalyzer(K8sClient(fc)).analyze_pod_communication("default/nope", "default/redis-0")


def test_deny_policy_blocks_ping(fc):
    fc.deny_ingress("default", {"app": "nginx"})
    t = RTTTester(K8sClient(fc)).test_pod_connectivity("default/frontend-5c7d8f9b4-kq2lp",
                                                      "default/nginx-web-6d4cf56db6-8v2mz")
    assert t.rtt_results[0].method == "ping" and not t.rtt_results[0].success
