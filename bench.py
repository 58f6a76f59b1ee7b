#!/usr/bin/env python
"""Headline benchmark: diagnostic queries/sec + p50 answer latency, Llama-3-8B TP=1, on the
``/api/v1/query`` path (BASELINE.json "metric").

One process per GPU (torchrun launches N ranks); each rank is an independent TP=1 engine replica
(data-parallel serving, weak scaling: per-GPU work is fixed).  One *step* = one wave of
``--batch`` concurrent diagnostic queries per GPU, each a synthetic cluster-state prompt in the
reference's prompt format answered with up to ``--max-new-tokens`` tokens through the
continuous-batching engine (prefill + hipGraph decode + sampling).  With ``--path http`` (default)
every query is a real ``POST /api/v1/query`` to the in-process REST server, sent by a child
load-generator process (``--client process``, default: remote clients do not share the serving
process's interpreter lock; ``--client thread`` keeps them in-process); ``--path engine``
submits to the engine queue directly (same engine, no HTTP).

Timing: W untimed warmup waves, then a barrier + device sync, K timed waves, a device sync + barrier;
the elapsed time is the MAX over ranks.  ``value`` = total queries answered by all ranks / that
time.  Weights are random-init (no checkpoints offline), prompts are synthetic (``data``).
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--model", default="llama-3-8b")
    ap.add_argument("--batch", type=int, default=64, help="concurrent queries per GPU per step")
    ap.add_argument("--max-new-tokens", type=int, default=256)
    ap.add_argument("--kv-cache-gb", type=float, default=48.0)
    ap.add_argument("--max-prefill-tokens", type=int, default=16384, help="token budget of one prefill step")
    ap.add_argument("--chunked-prefill", type=int, default=1, choices=[0, 1])
    ap.add_argument("--admit-gap-ms", type=float, default=None, help="engine admission coalescing gap (0 disables)")
    ap.add_argument("--admit-window-ms", type=float, default=None)
    ap.add_argument("--path", choices=["http", "engine", "podcomm"], default="http",
                    help="http: POST /api/v1/query (headline); podcomm: POST /api/v1/analyze/pod-communication "
                         "with the LLM explanation (BASELINE config 3); engine: the engine queue directly")
    ap.add_argument("--client", choices=["process", "thread"], default="process",
                    help="process: the HTTP clients run in a child load-generator process (remote clients; the "
                         "serving process keeps its interpreter lock); thread: client threads in this process")
    ap.add_argument("--no-graphs", action="store_true")
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--out", default=None, help="also write the JSON line to this file")
    a = ap.parse_args()

    loadgen = None
    if a.path in ("http", "podcomm") and a.client == "process":
        # started before this process initialises the GPU (the child never touches it)
        from k8s_llm_monitor_amd.monitor.loadgen import LoadGen

        loadgen = LoadGen(ROOT)

    import torch

    from k8s_llm_monitor_amd.engine import EngineConfig, EngineService, LLMEngine, SamplingParams
    from k8s_llm_monitor_amd.llm.synthetic import synthetic_cluster_prompt, synthetic_context
    from k8s_llm_monitor_amd.parallel import comm
    from k8s_llm_monitor_amd.parallel.state import barrier_all, init_parallel

    ps = init_parallel(tp_size=1)
    rank, world = ps.rank, ps.world_size
    if a.gpus != world and world > 1:
        print(f"warning: --gpus {a.gpus} but WORLD_SIZE {world}", file=sys.stderr)
    on_gpu = ps.device.type == "cuda"
    if on_gpu:
        from k8s_llm_monitor_amd import ops
        ops.native()  # fail loudly if the HIP kernels are missing

    admit = {k: v for k, v in (("admit_gap_ms", a.admit_gap_ms), ("admit_window_ms", a.admit_window_ms))
             if v is not None}
    eng = LLMEngine(EngineConfig(model=a.model, max_num_seqs=a.batch, max_model_len=8192, **admit,
                                 max_prefill_tokens=a.max_prefill_tokens, chunked_prefill=bool(a.chunked_prefill),
                                 kv_cache_gb=a.kv_cache_gb if on_gpu else 0.05, use_graphs=not a.no_graphs,
                                 seed=a.seed + rank), pstate=ps)
    eng.warmup()
    svc = EngineService(eng)
    server = None
    if a.path in ("http", "podcomm"):
        from k8s_llm_monitor_amd.monitor.app import build_app_for_bench

        server, port = build_app_for_bench(svc)
    params = SamplingParams(max_tokens=a.max_new_tokens, temperature=0.1, ignore_eos=True)

    def wave(w: int) -> tuple[list[float], int, int]:
        seeds = [rank * 1_000_003 + w * a.batch + i for i in range(a.batch)]
        if a.path == "http":
            from k8s_llm_monitor_amd.monitor.app import post_queries

            items = [synthetic_context(s)[::-1] for s in seeds]  # (question, cluster context)
            res = (loadgen.post_queries if loadgen else post_queries)(port, items, a.max_new_tokens)
            lat = [r["http_latency_ms"] for r in res]
            ptok = sum(r["prompt_tokens"] for r in res)
            gtok = sum(r["completion_tokens"] for r in res)
        elif a.path == "podcomm":
            from k8s_llm_monitor_amd.monitor.app import bench_pod_pairs, post_pod_communication

            pairs = bench_pod_pairs(a.batch * (w + 1))[a.batch * w:]
            res = (loadgen.post_pod_communication if loadgen else post_pod_communication)(port, pairs,
                                                                                          a.max_new_tokens)
            lat = [r["http_latency_ms"] for r in res]
            ptok = sum(r["prompt_tokens"] for r in res)
            gtok = sum(r["completion_tokens"] for r in res)
        else:
            futs = [svc.submit(synthetic_cluster_prompt(s), params) for s in seeds]
            outs = [f.result() for f in futs]
            lat = [s.timings()["latency_ms"] for _, s in outs]
            ptok = sum(len(s.prompt_ids) for _, s in outs)
            gtok = sum(len(s.output_ids) for _, s in outs)
        return lat, ptok, gtok

    for w in range(a.warmup):
        wave(w)
    barrier_all()
    if on_gpu:
        torch.cuda.synchronize()
    t0 = time.perf_counter()
    lats, ptoks, gtoks = [], 0, 0
    for k in range(a.steps):
        lat, p, g = wave(a.warmup + k)
        lats += lat
        ptoks += p
        gtoks += g
    if on_gpu:
        torch.cuda.synchronize()
    barrier_all()
    elapsed = time.perf_counter() - t0
    t_max = comm.all_reduce_max_scalar(elapsed)
    total_q = comm.all_reduce_sum_scalar(float(a.batch * a.steps))
    total_gen = comm.all_reduce_sum_scalar(float(gtoks))
    p50_local = statistics.median(lats)
    p50 = comm.all_reduce_max_scalar(p50_local)
    stats = svc.stats()
    if eng.trace is not None and rank == 0:
        _print_trace(eng.trace, t0)
    svc.close()
    if server is not None:
        server.shutdown()
    if loadgen is not None:
        loadgen.close()
    if rank == 0:
        qps = total_q / t_max
        name = _MODEL_NAMES.get(a.model, a.model)
        metric = (f"pod-communication analyses/sec ({name} TP=1, /api/v1/analyze/pod-communication)"
                  if a.path == "podcomm" else f"diagnostic queries/sec ({name} TP=1, /api/v1/query)")
        res = {
            "metric": metric,
            "value": round(qps, 4),
            "unit": "queries/s",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": round(t_max / a.steps * 1e3, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "bf16",
            "data": "synthetic cluster-state prompts (reference prepareLLMContext format), random-init weights",
            "config": {"model": a.model, "global_batch": a.batch * world, "seq_len": 8192,
                       "parallelism": f"dp{world}" if world > 1 else "tp1",
                       "prompt_tokens_mean": round(ptoks / max(1, a.batch * a.steps), 1),
                       "max_new_tokens": a.max_new_tokens, "path": a.path,
                       "client": a.client if a.path != "engine" else None},
            "p50_latency_ms": round(p50, 2),
            "p99_latency_ms": round(sorted(lats)[min(len(lats) - 1, int(len(lats) * 0.99))], 2),
            "generated_tokens_per_s": round(total_gen / t_max, 1),
            "decode_steps": stats.get("decode_steps"),
            "prefill_steps": stats.get("prefill_steps"),
        }
        line = json.dumps(res)
        print(line, flush=True)
        if a.out:
            with open(a.out, "w") as f:
                f.write(line + "\n")


_MODEL_NAMES = {"llama-3-8b": "Llama-3-8B", "llama-3-70b": "Llama-3-70B", "mixtral-8x7b": "Mixtral-8x7B",
                "gpt2-small": "GPT-2-small"}


def _print_trace(trace: list, t0: float) -> None:
    """K8SLLM_TRACE=1: per timed wave, when requests arrived, the prefill batches and the decode
    span (stderr)."""
    ev = [e for e in trace if e[0] >= t0]
    adds = [e for e in ev if e[1] == "add"]
    pre = [e for e in ev if e[1] == "prefill"]
    dec = [e for e in ev if e[1] == "decode"]
    if not adds:
        return
    waves, cur = [], [adds[0]]
    for e in adds[1:]:  # a new wave starts after a > 0.5 s pause in arrivals
        if e[0] - cur[-1][0] > 0.5:
            waves.append(cur)
            cur = []
        cur.append(e)
    waves.append(cur)
    subs = [e[0] for e in ev if e[1] == "submit"]
    if subs:
        print(f"[trace] submits {len(subs)}: " + " ".join(f"{(t - t0) * 1e3:.0f}" for t in subs[:200]), file=sys.stderr)
        print("[trace] adds: " + " ".join(f"{(e[0] - t0) * 1e3:.0f}" for e in adds[:200]), file=sys.stderr)
    for w in waves:
        gaps = sorted(b[0] - a_[0] for a_, b in zip(w, w[1:]))
        print(f"[trace] adds {len(w)} first +{(w[0][0] - t0) * 1e3:.1f} ms last +{(w[-1][0] - t0) * 1e3:.1f} ms"
              + (f" median gap {gaps[len(gaps) // 2] * 1e3:.2f} ms max gap {gaps[-1] * 1e3:.2f} ms" if gaps else ""),
              file=sys.stderr)
    for e in pre:
        print(f"[trace] prefill +{(e[0] - t0) * 1e3:.1f} ms seqs {e[2]} tokens {e[3]}", file=sys.stderr)
    if dec:
        print(f"[trace] decode steps {len(dec)} first +{(dec[0][0] - t0) * 1e3:.1f} last +{(dec[-1][0] - t0) * 1e3:.1f} ms",
              file=sys.stderr)


if __name__ == "__main__":
    main()
