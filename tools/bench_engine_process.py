#!/usr/bin/env python
"""The headline workload (64 concurrent /api/v1/query, ~1.6k-token prompts, 256 tokens, closed-loop
waves from the out-of-process load generator) served two ways on one GPU:

  * ``--mode inproc``: the engine thread shares the HTTP server's interpreter (bench.py's form);
  * ``--mode process``: the engine runs in a spawned child process behind ``engine.dp.ReplicaRouter``
    (one replica) - the HTTP handler threads of a wave's arrival burst no longer compete with the
    engine thread for the interpreter lock (profiles/r05/README.md "The wave boundary").

    python tools/bench_engine_process.py --mode process [--steps 5 --warmup 2]

Prints one JSON line: mode, queries/s over the timed waves, ms per wave."""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--mode", choices=["inproc", "process"], default="inproc")
    ap.add_argument("--model", default="llama-3-8b")
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--max-new-tokens", type=int, default=256)
    ap.add_argument("--kv-cache-gb", type=float, default=48.0)
    ap.add_argument("--device", default="cuda:0")
    a = ap.parse_args()
    from k8s_llm_monitor_amd.monitor.loadgen import LoadGen

    lg = LoadGen(ROOT)  # before anything touches the GPU
    from k8s_llm_monitor_amd.engine import EngineConfig

    cfg = EngineConfig(model=a.model, max_num_seqs=a.batch, max_model_len=8192, kv_cache_gb=a.kv_cache_gb, seed=0)
    if a.mode == "process":
        from k8s_llm_monitor_amd.engine.dp import ReplicaRouter

        svc = ReplicaRouter(cfg, [a.device])  # the child builds, warms up and captures its engine
    else:
        from k8s_llm_monitor_amd.engine import EngineService, LLMEngine

        eng = LLMEngine(cfg, device=a.device)
        eng.warmup()
        svc = EngineService(eng, max_queue=max(4 * a.batch, 256))
    from k8s_llm_monitor_amd.llm.synthetic import synthetic_context
    from k8s_llm_monitor_amd.monitor.app import build_app_for_bench

    server, port = build_app_for_bench(svc)
    n = a.batch
    for w in range(a.warmup + a.steps):
        lg.stage(w, [synthetic_context(w * n + i)[::-1] for i in range(n)])
    for w in range(a.warmup):
        lg.post_queries(port, None, a.max_new_tokens, slim=True, staged=w)
    t0 = time.perf_counter()
    res = lg.post_waves(port, list(range(a.warmup, a.warmup + a.steps)), a.max_new_tokens, slim=True)
    dt = time.perf_counter() - t0
    ok = sum(1 for r in res if r.get("http_status") == 200)
    print(json.dumps({"mode": a.mode, "queries_per_s": round(ok / dt, 4), "ms_per_wave": round(dt / a.steps * 1e3, 2),
                      "answered": ok, "waves": a.steps}), flush=True)
    server.shutdown()
    svc.close()
    lg.close()


if __name__ == "__main__":
    main()
