"""``test-k8s`` smoke CLI (cmd/test-k8s/main.go:44-185): connect, print cluster info, pods,
services, warning events, analyse the first two pods, then watch for 10 s (the reference's watch
returns immediately; this one really waits).  ``--fake`` runs against the FakeCluster."""
from __future__ import annotations

import argparse
import sys
import time

from ..monitor.cluster.client import K8sClient
from ..monitor.cluster.watch import EventHandler, ResourceWatcher
from ..monitor.config import from_dict, load


class CountingHandler(EventHandler):
    def __init__(self):
        self.pods = self.services = self.events = self.crds = 0

    def on_pod_update(self, pod):
        self.pods += 1
        print(f"  [watch] pod {pod.namespace}/{pod.name} -> {pod.status}")

    def on_service_update(self, svc):
        self.services += 1

    def on_event(self, ev):
        self.events += 1
        print(f"  [watch] event {ev.type} {ev.reason}: {ev.message}")

    def on_crd_event(self, ev):
        self.crds += 1


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(prog="test-k8s")
    ap.add_argument("-config", "--config", default="")
    ap.add_argument("--fake", action="store_true", help="use the deterministic FakeCluster")
    ap.add_argument("--watch-seconds", type=float, default=10.0)
    a = ap.parse_args(argv)
    cfg = load(a.config) if a.config else from_dict({"k8s": {"watch_namespaces": "default,kube-system"}})
    if a.fake:
        from ..monitor.cluster.fake import FakeCluster

        backend = FakeCluster.build()
    else:
        from ..monitor.app import make_backend

        backend = make_backend(cfg)
        if backend is None:
            print("no cluster configuration found (use --fake)")
            return 1
    c = K8sClient(backend, cfg.k8s)
    print("== connection:", c.test_connection())
    print("== cluster info:", c.get_cluster_info())
    pods = []
    for ns in c.namespaces:
        for p in c.get_pods(ns) or []:
            pods.append(p)
            print(f"  pod {p.namespace}/{p.name} {p.status} node={p.node_name} ip={p.ip}")
        for s in c.get_services(ns) or []:
            print(f"  svc {s.namespace}/{s.name} {s.type} {s.cluster_ip} selector={s.selector}")
        for e in c.get_events(ns, 20) or []:
            if e.type == "Warning":
                print(f"  warning {e.reason}: {e.message}")
    if len(pods) >= 2:
        from ..monitor.analysis.network import NetworkAnalyzer

        r = NetworkAnalyzer(c).analyze_pod_communication(f"{pods[0].namespace}/{pods[0].name}",
                                                         f"{pods[1].namespace}/{pods[1].name}")
        print(f"== analysis {r.pod_a} -> {r.pod_b}: {r.status} ({r.confidence}) issues={r.issues}")
    h = CountingHandler()
    w = ResourceWatcher(c, h, backoff_s=1.0, watch_timeout_s=max(1.0, a.watch_seconds))
    w.start()
    if a.fake:
        time.sleep(0.3)
        backend.crashloop_pod("default", "busybox-test", restarts=6)
    time.sleep(a.watch_seconds)
    w.stop()
    print(f"== watched: pods={h.pods} services={h.services} events={h.events}")
    return 0


if __name__ == "__main__":
    sys.exit(main())
