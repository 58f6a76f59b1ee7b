#!/usr/bin/env python
"""cProfile of one /api/v1/query request's host work through MonitorApp.handle (no sockets, no
GPU): request parse, context fit, prompt build, tokenization, response encoding - against the
instant engine stand-in of tools/bench_http_wave.py.

    python tools/profile_query_path.py [--n 200 --top 25]"""
from __future__ import annotations

import argparse
import cProfile
import json
import os
import pstats
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=200)
    ap.add_argument("--top", type=int, default=25)
    a = ap.parse_args()
    from bench_http_wave import InstantService

    from k8s_llm_monitor_amd.llm.synthetic import synthetic_context
    from k8s_llm_monitor_amd.monitor.app import build_app_for_bench

    svc = InstantService(1, 256)
    srv, _ = build_app_for_bench(svc)
    app = srv.RequestHandlerClass.app if hasattr(srv.RequestHandlerClass, "app") else None
    if app is None:
        raise SystemExit("cannot reach the MonitorApp from the server")
    bodies = []
    for s in range(a.n):
        q, ctx = synthetic_context(s)[::-1]
        bodies.append(json.dumps({"question": q, "max_tokens": 256, "ignore_eos": True,
                                  "context": {"cluster_state": ctx}}).encode())
    for b in bodies[:5]:
        app.handle("POST", "/api/v1/query", b)
    t = time.perf_counter()
    pr = cProfile.Profile()
    pr.enable()
    for b in bodies:
        r = app.handle("POST", "/api/v1/query", b)
    pr.disable()
    dt = (time.perf_counter() - t) / a.n
    print(f"per request (profiled): {dt * 1e3:.3f} ms; last status {getattr(r, 'status', '?')}")
    pstats.Stats(pr).sort_stats("cumulative").print_stats(a.top)
    # the part that runs on the server's worker pool: AnalysisService.query (context fit, prompt,
    # tokenization, submit) in this thread
    items = [synthetic_context(s)[::-1] for s in range(a.n)]
    pr = cProfile.Profile()
    t = time.perf_counter()
    pr.enable()
    for q, ctx in items:
        app.analysis.query(q, max_tokens=256, ignore_eos=True, context_text=ctx)
    pr.disable()
    print(f"AnalysisService.query per request (profiled): {(time.perf_counter() - t) / a.n * 1e3:.3f} ms")
    pstats.Stats(pr).sort_stats("cumulative").print_stats(a.top)
    srv.shutdown()


if __name__ == "__main__":
    main()
