"""HTTP smoke checks against a running monitor server - the checks of the reference's
``test_server.sh``, ``test_with_mock_k8s.sh``, ``test_web_interface.sh`` and
``scripts/test_uav_collection.sh`` as one stdlib-only tool (no curl/jq needed).

    python tools/smoke.py server [--url http://127.0.0.1:8080]   # health, status, pods, errors, query, web UI
    python tools/smoke.py uav    [--url ...] [--push]             # UAV metrics, per-node, CRDs, push report

Exit status is the number of failed checks (0 = all passed).  ``scripts/*.sh`` wrap this.
"""
from __future__ import annotations

import argparse
import json
import sys
import time
import urllib.error
import urllib.request
from typing import Any, Callable, Optional


class Smoke:
    def __init__(self, url: str, verbose: bool = True):
        self.url = url.rstrip("/")
        self.verbose = verbose
        self.failed: list[str] = []
        self.passed: list[str] = []

    def req(self, method: str, path: str, body: Any = None, timeout: float = 30.0) -> tuple[int, Any, str]:
        data = json.dumps(body).encode() if body is not None else None
        r = urllib.request.Request(self.url + path, data=data, method=method,
                                   headers={"Content-Type": "application/json"} if data else {})
        try:
            with urllib.request.urlopen(r, timeout=timeout) as resp:
                raw = resp.read().decode("utf-8", "replace")
                code = resp.status
        except urllib.error.HTTPError as e:
            raw = e.read().decode("utf-8", "replace")
            code = e.code
        try:
            return code, json.loads(raw), raw
        except ValueError:
            return code, None, raw

    def check(self, name: str, fn: Callable[[], Optional[str]]) -> None:
        try:
            err = fn()
        except Exception as e:  # noqa: BLE001 - a smoke check reports, it does not crash
            err = f"{type(e).__name__}: {e}"
        (self.failed if err else self.passed).append(name)
        if self.verbose:
            print(("  ok   " if not err else "  FAIL ") + name + ("" if not err else f"  ({err})"), flush=True)

    # ------------------------------------------------------------------ suites
    def server_suite(self, query: bool = True) -> None:
        def health():
            c, j, _ = self.req("GET", "/health")
            return None if c == 200 and j and j.get("status") == "healthy" else f"{c} {j}"

        def status():
            c, j, _ = self.req("GET", "/api/v1/cluster/status")
            return None if c == 200 and j and "status" in j else f"{c} {j}"

        def pods():
            c, j, _ = self.req("GET", "/api/v1/pods")
            return None if c == 200 and j and isinstance(j.get("count"), int) else f"{c} {j}"

        def bad_request():
            c, _, _ = self.req("POST", "/api/v1/analyze/pod-communication", {"invalid": "data"})
            return None if c == 400 else f"expected 400, got {c}"

        def pod_comm():
            c, j, _ = self.req("GET", "/api/v1/pods")
            names = [f"{p['namespace']}/{p['name']}" for p in (j or {}).get("pods", [])][:2]
            if len(names) < 2:
                return None  # nothing to pair (real cluster with < 2 pods): not a failure
            c, j, _ = self.req("POST", "/api/v1/analyze/pod-communication", {"pod_a": names[0], "pod_b": names[1]})
            return None if c == 200 and j and "status" in j else f"{c} {j}"

        def metrics():
            for p in ("/api/v1/metrics/cluster", "/api/v1/metrics/nodes", "/api/v1/metrics/pods"):
                c, _, _ = self.req("GET", p)
                if c not in (200, 503):
                    return f"{p}: {c}"
            return None

        def ask():
            c, j, _ = self.req("POST", "/api/v1/query", {"question": "Which pods are unhealthy and why?",
                                                         "max_tokens": 32}, timeout=300)
            return None if c == 200 and j and j.get("status") == "success" else f"{c} {j}"

        def web():
            c, _, raw = self.req("GET", "/")
            return None if c == 200 and "K8s LLM Monitor" in raw else f"{c}, title missing"

        self.check("health", health)
        self.check("cluster status", status)
        self.check("pod list", pods)
        self.check("error handling (400 on invalid body)", bad_request)
        self.check("pod communication analysis", pod_comm)
        self.check("metrics endpoints", metrics)
        if query:
            self.check("POST /api/v1/query", ask)
        self.check("web console", web)

    def uav_suite(self, push: bool = True) -> None:
        state: dict = {}

        def uav_list():
            c, j, _ = self.req("GET", "/api/v1/metrics/uav")
            if c != 200 or j is None:
                return f"{c} {j}"
            state["uavs"] = j.get("uavs") or j.get("data") or {}
            return None

        def uav_push():
            rep = {"node_name": "smoke-node", "uav_id": "UAV-smoke-node",
                   "timestamp": time.strftime("%Y-%m-%dT%H:%M:%SZ", time.gmtime()),
                   "state": {"uav_id": "UAV-smoke-node", "node_name": "smoke-node",
                             "battery": {"remaining_percent": 77.0, "voltage": 15.8},
                             "gps": {"latitude": 39.9, "longitude": 116.4, "altitude": 50.0, "satellite_count": 12,
                                     "fix_type": 3},
                             "flight": {"mode": "LOITER", "armed": True},
                             "health": {"system_status": "OK"}},
                   "heartbeat_interval_seconds": 10}
            c, j, _ = self.req("POST", "/api/v1/uav/report", rep)
            return None if c == 200 else f"{c} {j}"

        def uav_node():
            c, j, _ = self.req("GET", "/api/v1/metrics/uav/smoke-node")
            return None if c == 200 and j else f"{c} {j}"

        def battery_gps():
            c, j, _ = self.req("GET", "/api/v1/metrics/uav")
            blob = json.dumps(j)
            return None if c == 200 and "battery" in blob and "gps" in blob else "no battery/gps fields"

        def crds():
            c, j, _ = self.req("GET", "/api/v1/crd/uav")
            return None if c in (200, 503) else f"{c} {j}"

        def states() -> dict:
            c, j, _ = self.req("GET", "/api/v1/metrics/uav")
            data = (j or {}).get("data") or {}
            return {k: (v.get("state") or v) if isinstance(v, dict) else {} for k, v in data.items()}

        def single_from_list():  # reference test_get_single_uav: the first listed node
            st = states()
            if not st:
                return "no UAV listed"
            node = sorted(st)[0]
            c, j, _ = self.req("GET", f"/api/v1/metrics/uav/{node}")
            return None if c == 200 and (j or {}).get("status") == "success" else f"{node}: {c} {j}"

        def integrity():  # reference test_data_integrity: the five fields of the first entry
            st = states()
            if not st:
                return "no UAV listed"
            first = st[sorted(st)[0]]
            missing = [f for f in ("uav_id", "gps", "battery", "flight", "health") if first.get(f) is None]
            return f"missing fields {missing}" if missing else None

        def monitor(label, pred, fmt):
            """Reference low-battery / GPS / health monitors: list the offenders (a warning, as in
            the reference, not a failure)."""
            def run():
                bad = [fmt(k, v) for k, v in sorted(states().items()) if pred(v)]
                print(f"    {label}: " + ("none" if not bad else "; ".join(bad)))
                return None
            return run

        def latency():  # reference test_performance: average of 10 GETs, < 1000 ms good, > 3 s slow
            ts = []
            for _ in range(10):
                t0 = time.perf_counter()
                self.req("GET", "/api/v1/metrics/uav")
                ts.append((time.perf_counter() - t0) * 1e3)
            avg = sum(ts) / len(ts)
            grade = "good (<1s)" if avg < 1000 else ("fair (1-3s)" if avg < 3000 else "slow (>3s)")
            print(f"    average response {avg:.1f} ms: {grade}")
            return None if avg < 3000 else f"average {avg:.0f} ms"

        self.check("UAV metrics list", uav_list)
        if push:
            self.check("UAV report push", uav_push)
            self.check("UAV metrics by node", uav_node)
            self.check("UAV battery + GPS present", battery_gps)
        self.check("UAV single lookup (first listed node)", single_from_list)
        self.check("UAV data integrity (uav_id/gps/battery/flight/health)", integrity)
        self.check("low battery monitor (<20%)", monitor(
            "low battery", lambda v: float((v.get("battery") or {}).get("remaining_percent", 100)) < 20,
            lambda k, v: f"{k}: {v['battery']['remaining_percent']}%"))
        self.check("GPS monitor (<10 satellites)", monitor(
            "weak GPS", lambda v: int((v.get("gps") or {}).get("satellite_count", 99)) < 10,
            lambda k, v: f"{k}: {v['gps'].get('satellite_count')} satellites"))
        self.check("health monitor (system_status != OK)", monitor(
            "unhealthy", lambda v: (v.get("health") or {}).get("system_status", "OK") != "OK",
            lambda k, v: f"{k}: {v['health'].get('system_status')}"))
        self.check("collection latency (10 GETs)", latency)
        self.check("UAVMetric CRD list", crds)
        for k, v in sorted(states().items()):  # reference generate_report
            print(f"    {k}: battery {(v.get('battery') or {}).get('remaining_percent')}%, "
                  f"GPS {(v.get('gps') or {}).get('satellite_count')} sats, mode {(v.get('flight') or {}).get('mode')}, "
                  f"status {(v.get('health') or {}).get('system_status')}")


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__.split("\n\n")[0])
    ap.add_argument("suite", choices=["server", "uav", "all"])
    ap.add_argument("--url", default="http://127.0.0.1:8080")
    ap.add_argument("--no-query", action="store_true", help="skip POST /api/v1/query (no LLM backend)")
    ap.add_argument("--no-push", action="store_true")
    ap.add_argument("--wait", type=float, default=0.0, help="seconds to wait for /health first")
    a = ap.parse_args(argv)
    s = Smoke(a.url)
    deadline = time.time() + a.wait
    while a.wait and time.time() < deadline:
        try:
            if s.req("GET", "/health", timeout=2)[0] == 200:
                break
        except OSError:
            time.sleep(0.5)
    if a.suite in ("server", "all"):
        print("server checks:")
        s.server_suite(query=not a.no_query)
    if a.suite in ("uav", "all"):
        print("UAV collection checks:")
        s.uav_suite(push=not a.no_push)
    print(f"{len(s.passed)} passed, {len(s.failed)} failed")
    return len(s.failed)


if __name__ == "__main__":
    sys.exit(main())
