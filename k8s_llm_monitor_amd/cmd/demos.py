"""The reference's interactive demos (cmd/demos/*, B5-B9) as subcommands:

    python -m k8s_llm_monitor_amd.cmd.demos {crd,debug,live,network,rtt} [--fake] [...]
"""
from __future__ import annotations

import argparse
import sys
import time

from ..monitor.cluster.client import K8sClient
from ..monitor.config import from_dict


def _client(a) -> K8sClient:
    cfg = from_dict({"k8s": {"watch_namespaces": a.namespaces}})
    if a.fake:
        from ..monitor.cluster.fake import FakeCluster

        return K8sClient(FakeCluster.build(), cfg.k8s)
    from ..monitor.app import make_backend

    cfg.k8s.backend = "kube"
    return K8sClient(make_backend(cfg), cfg.k8s)


def crd_demo(a) -> None:
    from ..monitor.cluster.watch import CRDWatcher, EventHandler

    class H(EventHandler):
        def on_crd_event(self, ev):
            print(f"  CRD event {ev.type} {ev.group}/{ev.kind} {ev.namespace}/{ev.name}")

    c = _client(a)
    w = CRDWatcher(c, H(), backoff_s=1.0, watch_timeout_s=a.seconds)
    for crd in w.get_crds():
        print(f"CRD {crd.name}: kind={crd.kind} scope={crd.scope} versions={crd.versions} established={crd.established}")
    w.start()
    time.sleep(a.seconds)
    w.stop()


def debug_demo(a) -> None:
    c = _client(a)
    print("step 1 connection:", c.test_connection())
    print("step 2 cluster info:", c.get_cluster_info())
    for ns in c.namespaces:
        print(f"step 3 pods in {ns}:", [p.name for p in c.get_pods(ns) or []])
        print(f"step 4 services in {ns}:", [s.name for s in c.get_services(ns) or []])
        print(f"step 5 events in {ns}:", [(e.type, e.reason) for e in c.get_events(ns, 10) or []])


def live_demo(a) -> None:
    from .test_k8s import CountingHandler
    from ..monitor.cluster.watch import ResourceWatcher

    c = _client(a)
    w = ResourceWatcher(c, CountingHandler(), backoff_s=1.0, watch_timeout_s=a.seconds)
    w.start()
    t_end = time.time() + a.seconds
    while time.time() < t_end:
        n = sum(len(c.get_pods(ns) or []) for ns in c.namespaces)
        print(f"[{time.strftime('%H:%M:%S')}] pods: {n}")
        time.sleep(min(30.0, max(0.5, a.seconds / 3)))
    w.stop()


def network_demo(a) -> None:
    from ..monitor.analysis.network import NetworkAnalyzer

    c = _client(a)
    r = NetworkAnalyzer(c).analyze_pod_communication(a.pod_a, a.pod_b)
    print(f"{r.pod_a} -> {r.pod_b}: {r.status} confidence={r.confidence}")
    for i, s in zip(r.issues or [], r.solutions or []):
        print(f"  issue: {i}\n    fix: {s}")


def rtt_demo(a) -> None:
    from ..monitor.analysis.network import NetworkAnalyzer, RTTTester

    c = _client(a)
    r = RTTTester(c).test_pod_connectivity(a.pod_a, a.pod_b)
    for x in r.rtt_results or []:
        print(f"  {x.method}: success={x.success} rtt={x.rtt:.3f}ms loss={x.packet_loss}% {x.error_message}")
    print(f"avg={r.average_rtt:.3f}ms success={r.success_rate:.1f}% latency={r.latency}")
    network_demo(a)


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(prog="demos")
    ap.add_argument("demo", choices=["crd", "debug", "live", "network", "rtt"])
    ap.add_argument("--fake", action="store_true")
    ap.add_argument("--namespaces", default="default,kube-system")
    ap.add_argument("--seconds", type=float, default=5.0)
    ap.add_argument("--pod-a", default="default/busybox-test")
    ap.add_argument("--pod-b", default="default/nginx-web-6d4cf56db6-8v2mz")
    a = ap.parse_args(argv)
    {"crd": crd_demo, "debug": debug_demo, "live": live_demo, "network": network_demo, "rtt": rtt_demo}[a.demo](a)
    return 0


if __name__ == "__main__":
    sys.exit(main())
