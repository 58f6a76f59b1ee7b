import time

from k8s_llm_monitor_amd.monitor.cluster.backend import UAV_METRICS
from k8s_llm_monitor_amd.monitor.cluster.client import K8sClient
from k8s_llm_monitor_amd.monitor.cluster.fake import FakeCluster
from k8s_llm_monitor_amd.monitor.cluster.watch import CRDWatcher, EventHandler, ResourceWatcher
from k8s_llm_monitor_amd.monitor.config import K8sConfig
from k8s_llm_monitor_amd.monitor.types import UAVReport


class Rec(EventHandler):
    def __init__(self):
        self.pods, self.svcs, self.events, self.crd = [], [], [], []

    def on_pod_update(self, p):
        self.pods.append((p.name, p.status))

    def on_service_update(self, s):
        self.svcs.append(s.name)

    def on_event(self, e):
        self.events.append(e.reason)

    def on_crd_event(self, e):
        self.crd.append((e.type, e.kind, e.name))


def _wait(cond, t=5.0):
    end = time.time() + t
    while time.time() < end and not cond():
        time.sleep(0.05)
    return cond()


def test_resource_watcher_dispatch_and_idempotent_stop():
    fc = FakeCluster.build(seed=7)
    h = Rec()
    w = ResourceWatcher(K8sClient(fc, K8sConfig(watch_namespaces="default")), h, backoff_s=0.2, watch_timeout_s=2)
    w.start()
    assert _wait(lambda: len(h.pods) >= 5 and h.svcs)
    fc.fail_pod("default", "redis-0")
    assert _wait(lambda: ("redis-0", "Failed") in h.pods)
    assert _wait(lambda: "Error" in h.events)
    w.stop()
    w.stop()


def test_crd_watcher_cache():
    fc = FakeCluster.build(seed=7)
    c = K8sClient(fc)
    h = Rec()
    w = CRDWatcher(c, h, backoff_s=0.2, watch_timeout_s=2)
    assert {x.kind for x in w.get_crds()} == {"UAVMetric", "SchedulingRequest"}
    w.start()
    time.sleep(0.3)
    c.upsert_uav_metric(UAVReport(node_name="n9", uav_id="U9"))
    assert _wait(lambda: ("ADDED", "UAVMetric", "uavmetric-n9") in h.crd)
    assert _wait(lambda: [r.name for r in w.get_custom_resources("monitoring.io", "UAVMetric", "default")] == ["uavmetric-n9"])
    fc.delete(UAV_METRICS, "uavmetric-n9", "default")
    assert _wait(lambda: w.get_custom_resources("monitoring.io", "UAVMetric", "default") == [])
    w.stop()
