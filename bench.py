#!/usr/bin/env python
"""Headline benchmark: diagnostic queries/sec + p50 answer latency, Llama-3-8B TP=1, on the
``/api/v1/query`` path (BASELINE.json "metric").

Process model: one process per GPU.  ``python bench.py --gpus N`` launches N rank processes by
itself (before anything touches a GPU) when it is not already running under torchrun; under
``torch.distributed.run`` (the driver's multi-GPU command) each process is one rank.  Ranks form
``N / tp`` engine replicas (data parallel, weak scaling: per-replica work is fixed) of ``--tp``
GPUs each (tensor parallel over RCCL / the one-shot IPC all-reduce).  The TP leader of each
replica serves HTTP; its TP workers mirror its steps (parallel/step_bus.py).

Modes (``--mode``):
* ``wave`` (default, the headline) - one step = one closed-loop wave of ``--batch`` concurrent
  diagnostic queries per replica, each a synthetic cluster-state prompt in the reference's prompt
  format answered with ``--max-new-tokens`` tokens through the continuous-batching engine.
* ``poisson`` - open loop: ``--steps x --batch`` queries per replica arriving as a Poisson process
  at ``--rate`` queries/s; reports TTFT / TPOT / latency percentiles (mixed prefill+decode steps
  at work).
* ``latency`` - batch 1: one query at a time; a step = one query.
``--production``: the server runs with the reference's timeouts (15 s write, 30 s llm.timeout)
instead of the bench's 600 s; answers that reach the deadline come back truncated
(finish_reason "deadline") and overload as 503 - both are counted in the JSON line.

With ``--path http`` (default) every query is a real ``POST /api/v1/query`` to the in-process REST
server, sent by a child load-generator process (``--client process``); ``--path engine`` submits
to the engine queue directly; ``--path podcomm`` posts /api/v1/analyze/pod-communication.

Weights: one resident copy in the decode kernels' packed layout, read by prefill too (default
``--layout one``; ``--layout two`` = the round-5 row-major weights + decode copies, for A/B runs);
the JSON config reports the layout and the resident weight GB per rank.

Timing: W untimed warmup steps, then a barrier + device sync, K timed steps, a device sync +
barrier; the elapsed time is the MAX over ranks.  ``value`` = total queries answered by all
replicas / that time.  Weights are random-init (no checkpoints offline), prompts are synthetic.
"""
from __future__ import annotations

import argparse
import json
import os
import random
import statistics
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

_MODEL_NAMES = {"llama-3-8b": "Llama-3-8B", "llama-3-70b": "Llama-3-70B", "mixtral-8x7b": "Mixtral-8x7B",
                "gpt2-small": "GPT-2-small"}


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1, help="ranks (one per GPU) of this node")
    ap.add_argument("--tp", type=int, default=1, help="tensor-parallel degree of one engine replica")
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--model", default="llama-3-8b")
    ap.add_argument("--batch", type=int, default=64, help="concurrent queries per replica per step")
    ap.add_argument("--max-new-tokens", type=int, default=256)
    ap.add_argument("--mode", choices=["wave", "poisson", "latency"], default="wave")
    ap.add_argument("--rate", type=float, default=16.0, help="poisson: arrivals per second per replica")
    ap.add_argument("--production", action="store_true",
                    help="reference server timeouts (15 s write / 30 s llm): deadline truncation + 503s")
    ap.add_argument("--kv-cache-gb", type=float, default=48.0)
    ap.add_argument("--max-prefill-tokens", type=int, default=16384, help="token budget of one prefill step")
    ap.add_argument("--mixed-prefill-tokens", type=int, default=None,
                    help="prefill budget of a mixed prefill+decode step (0: prefill stalls decodes)")
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
    ap.add_argument("--decode-fusion", choices=["auto", "none", "rc"], default="auto",
                    help="A/B runs of the decode-step fusion (CausalLM.set_decode_fusion): auto = the "
                         "default (row-complete o only for the smallest buckets), none = off, rc = "
                         "every bucket")
    ap.add_argument("--layout", choices=["one", "two"], default="one",
                    help="dense Llama weights: one = the single fragment-packed copy read by prefill and "
                         "decode (CausalLM.ONE_LAYOUT), two = row-major prefill weights + decode copies "
                         "(the round-5 form, for A/B runs)")
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--out", default=None, help="also write the JSON line to this file")
    a = ap.parse_args(argv)
    if a.mode == "latency":
        a.batch = 1
    if a.gpus < 1 or a.tp < 1 or a.gpus % a.tp:
        ap.error(f"--tp {a.tp} must divide --gpus {a.gpus}")
    return a


# --------------------------------------------------------------------------- launcher

def spawn_ranks(n: int, argv: list, timeout_s: float = 0.0) -> int:
    """Run this script as ``n`` rank processes (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* set, one
    GPU each) and return the first non-zero exit code (0 when all succeed).  Called before this
    process touches any GPU; rank 0's stdout (the JSON line) is this process's stdout.  A rank that
    fails takes the others down (they would otherwise wait in a collective forever).

    Rendezvous: this process hosts the ranks' TCP store itself, on a port the OS picks at bind time
    and that stays bound until the ranks are gone (K8SLLM_EXTERNAL_STORE tells init_parallel to
    join it as a client) - no probe-then-release window in which another process can take it."""
    import datetime

    from torch.distributed import TCPStore  # CPU only: does not initialise the GPU

    store = TCPStore("127.0.0.1", 0, n + 1, is_master=True, timeout=datetime.timedelta(seconds=600),
                     wait_for_workers=False)
    port = store.port
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), K8SLLM_EXTERNAL_STORE="1")
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__), *argv], env=env,
                                      start_new_session=True))
    t0 = time.time()
    rc = 0
    try:
        while True:
            codes = [p.poll() for p in procs]
            bad = [c for c in codes if c not in (None, 0)]
            if bad:
                rc = bad[0]
                break
            if all(c == 0 for c in codes):
                break
            if timeout_s and time.time() - t0 > timeout_s:
                rc = 124
                break
            time.sleep(0.2)
    finally:
        for p in procs:
            if p.poll() is None:
                try:
                    os.killpg(p.pid, 15)
                except ProcessLookupError:
                    pass
        for p in procs:
            try:
                p.wait(timeout=30)
            except subprocess.TimeoutExpired:
                os.killpg(p.pid, 9)
                p.wait()
    return rc


# --------------------------------------------------------------------------- one rank

def _pct(xs: list, q: float):
    if not xs:
        return None
    xs = sorted(xs)
    return round(xs[min(len(xs) - 1, int(len(xs) * q))], 2)


def run_rank(a) -> None:
    env_rank = int(os.environ.get("RANK", "0"))
    leader = env_rank % a.tp == 0
    loadgen = None
    if leader and a.path in ("http", "podcomm") and a.client == "process":
        # started before this process initialises the GPU (the child never touches it)
        from k8s_llm_monitor_amd.monitor.loadgen import LoadGen

        loadgen = LoadGen(ROOT)

    import torch
    import torch.distributed as dist

    from k8s_llm_monitor_amd.engine import EngineConfig, EngineService, LLMEngine, SamplingParams
    from k8s_llm_monitor_amd.llm.synthetic import synthetic_cluster_prompt, synthetic_context
    from k8s_llm_monitor_amd.parallel import comm
    from k8s_llm_monitor_amd.parallel.state import init_parallel

    ps = init_parallel(tp_size=a.tp)
    rank, world = ps.rank, ps.world_size
    if a.gpus != world:
        print(f"warning: --gpus {a.gpus} but WORLD_SIZE {world}", file=sys.stderr)
    dp = world // a.tp
    on_gpu = ps.device.type == "cuda"
    if on_gpu:
        from k8s_llm_monitor_amd import ops

        ops.native()  # fail loudly if the HIP kernels are missing
    # the replicas' leaders synchronise the timed region among themselves (workers are inside
    # worker_loop); every rank creates the group, in the same order
    leaders_group = None
    if world > 1:
        leaders_group = dist.new_group(list(range(0, world, a.tp)), backend="gloo")

    def leaders_barrier() -> None:
        if leaders_group is not None:
            dist.barrier(group=leaders_group)

    admit = {k: v for k, v in (("admit_gap_ms", a.admit_gap_ms), ("admit_window_ms", a.admit_window_ms),
                               ("mixed_prefill_tokens", a.mixed_prefill_tokens)) if v is not None}
    if not on_gpu:
        # the CPU engine's steps are seconds long and its HTTP handlers share the same 8 cores, so a
        # wave's requests arrive over ~100 ms: coalesce them for 250 ms (still ~1/8 of one CPU
        # prefill step) so the wave starts as one prefill batch (config 1, VERDICT r5 Missing #3)
        admit.setdefault("admit_gap_ms", 25.0)
        admit.setdefault("admit_window_ms", 250.0)
    from k8s_llm_monitor_amd.models.llama import CausalLM
    CausalLM.ONE_LAYOUT = a.layout == "one"
    eng = LLMEngine(EngineConfig(model=a.model, max_num_seqs=max(a.batch, 8) if a.mode == "latency" else a.batch,
                                 max_model_len=8192, max_prefill_tokens=a.max_prefill_tokens,
                                 chunked_prefill=bool(a.chunked_prefill), tp_size=a.tp,
                                 kv_cache_gb=a.kv_cache_gb if on_gpu else 0.0, use_graphs=not a.no_graphs,
                                 seed=a.seed + ps.dp_rank, **admit), pstate=ps)
    if a.decode_fusion != "auto":
        eng.model.set_decode_fusion(rc=a.decode_fusion == "rc")
    eng.warmup()
    devices = [str(ps.device)] * world
    if world > 1:
        dist.all_gather_object(devices, str(ps.device))

    if not ps.tp_leader:  # TP worker: mirror the leader's steps, then join the final reductions
        eng.worker_loop()
        _finish(a, ps, comm, 0.0, 0, 0, 0, [], {}, devices, eng, on_gpu)
        return

    svc = EngineService(eng, max_queue=max(4 * a.batch, 256))
    server = port = None
    if a.path in ("http", "podcomm"):
        from k8s_llm_monitor_amd.monitor.app import build_app_for_bench

        tmo = dict(write_timeout_s=15.0, llm_timeout_s=30.0) if a.production else {}
        server, port = build_app_for_bench(svc, **tmo)
    params = SamplingParams(max_tokens=a.max_new_tokens, temperature=0.1, ignore_eos=True)
    rng = random.Random(1234 + ps.dp_rank)

    def post(w, items, offsets=None):
        from k8s_llm_monitor_amd.monitor.app import post_queries

        kw = dict(offsets_s=offsets, allow_errors=a.production or a.mode == "poisson")
        if loadgen:
            return loadgen.post_queries(port, None, a.max_new_tokens, slim=True, staged=w, **kw)
        return post_queries(port, items, a.max_new_tokens, **kw)

    # the clients' synthetic payloads are generated up front: building them is load-generator
    # work (~13 ms per 64-query wave), not serving work, so it stays out of the timed region
    n = a.batch
    seeds_of = {w: [ps.dp_rank * 1_000_003 + w * n + i for i in range(n)] for w in range(a.warmup + a.steps)}
    payload = {}
    if a.path == "http":
        payload = {w: [synthetic_context(sd)[::-1] for sd in seeds_of[w]] for w in seeds_of}  # (question, context)
        if loadgen:  # the clients hold their payloads before the clock starts: per wave only a key crosses the pipe
            for w, items in payload.items():
                loadgen.stage(w, items)
    elif a.path == "engine":
        payload = {w: [synthetic_cluster_prompt(sd) for sd in seeds_of[w]] for w in seeds_of}

    def step(w: int) -> list[dict]:
        """One bench step; per-request result dicts (http_status, latency_ms, ttft_ms, tokens)."""
        if a.path == "http":
            items = payload[w]
            if a.mode == "poisson":
                t, offs = 0.0, []
                for _ in items:
                    t += rng.expovariate(a.rate)
                    offs.append(t)
                return post(w, items, offs)
            return post(w, items)
        if a.path == "podcomm":
            from k8s_llm_monitor_amd.monitor.app import bench_pod_pairs, post_pod_communication

            pairs = bench_pod_pairs(n * (w + 1))[n * w:]
            return (loadgen.post_pod_communication if loadgen else post_pod_communication)(port, pairs,
                                                                                          a.max_new_tokens)
        futs = [svc.submit(prompt, params) for prompt in payload[w]]
        out = []
        for f in futs:
            _, s = f.result()
            d = s.timings()
            d.update(http_status=200, http_latency_ms=d["latency_ms"], finish_reason=s.finish_reason)
            out.append(d)
        return out

    # progress heartbeat on stderr (a long wave otherwise prints nothing for minutes)
    import threading

    hb_stop = threading.Event()

    def heartbeat() -> None:
        t_hb = time.perf_counter()
        while not hb_stop.wait(30.0):
            c = eng.counters
            print(f"[bench] rank {rank} +{time.perf_counter() - t_hb:.0f}s prefill {c['prefill_steps']} "
                  f"decode {c['decode_steps']} mixed {c['mixed_steps']}", file=sys.stderr, flush=True)

    threading.Thread(target=heartbeat, daemon=True, name="bench-heartbeat").start()
    for w in range(a.warmup):
        step(w)
    leaders_barrier()
    if on_gpu:
        torch.cuda.synchronize()
    t0 = time.perf_counter()
    res: list[dict] = []
    if loadgen and a.path == "http" and a.mode == "wave":
        # the K closed-loop waves run inside the client process (wave k+1 goes out when wave k is
        # answered, as step() does per wave) - no parent <-> client pipe round trip between waves
        res = loadgen.post_waves(port, list(range(a.warmup, a.warmup + a.steps)), a.max_new_tokens,
                                 allow_errors=a.production, slim=True)
    else:
        for k in range(a.steps):
            res += step(a.warmup + k)
    if on_gpu:
        torch.cuda.synchronize()
    leaders_barrier()
    elapsed = time.perf_counter() - t0
    hb_stop.set()
    ok = [r for r in res if r.get("http_status", 200) == 200]
    stats = svc.stats()
    if eng.trace is not None and rank == 0:
        _print_trace(eng.trace, t0)
    svc.close()  # stops this replica's TP workers
    if server is not None:
        server.shutdown()
    if loadgen is not None:
        loadgen.close()
    ptoks = sum(r.get("prompt_tokens", 0) for r in ok)
    gtoks = sum(r.get("completion_tokens", 0) for r in ok)
    # `value` counts complete answers: a production-mode answer cut at its deadline is reported
    # separately (requests.deadline_truncated_rank0), not as a served query
    n_full = sum(1 for r in ok if r.get("finish_reason") != "deadline")
    _finish(a, ps, comm, elapsed, n_full, ptoks, gtoks, res, stats, devices, eng, on_gpu, n_answered=len(ok))


def _finish(a, ps, comm, elapsed, n_ok, ptoks, gtoks, res, stats, devices, eng, on_gpu, n_answered=None) -> None:
    world = ps.world_size
    t_max = comm.all_reduce_max_scalar(elapsed)
    total_q = comm.all_reduce_sum_scalar(float(n_ok))
    # prompt tokens are summed over every answered request (deadline-truncated ones included)
    total_ans = comm.all_reduce_sum_scalar(float(n_ok if n_answered is None else n_answered))
    total_gen = comm.all_reduce_sum_scalar(float(gtoks))
    total_p = comm.all_reduce_sum_scalar(float(ptoks))
    ok = [r for r in res if r.get("http_status", 200) == 200]
    lats = [r["http_latency_ms"] for r in ok]
    p50 = comm.all_reduce_max_scalar(statistics.median(lats) if lats else 0.0)
    # the longest sequence served (prompt + answer tokens): the config's real seq_len
    seq_max = int(comm.all_reduce_max_scalar(float(max((r.get("prompt_tokens", 0) + r.get("completion_tokens", 0)
                                                        for r in ok), default=0))))
    if ps.rank != 0:
        return
    dp = world // a.tp
    name = _MODEL_NAMES.get(a.model, a.model)
    tp_s = f"TP={a.tp}"
    metric = (f"pod-communication analyses/sec ({name} {tp_s}, /api/v1/analyze/pod-communication)"
              if a.path == "podcomm" else f"diagnostic queries/sec ({name} {tp_s}, /api/v1/query)")
    if world == 1:
        par = "tp1"
    elif a.tp == 1:
        par = f"dp{dp}"
    elif dp == 1:
        par = f"tp{a.tp}"
    else:
        par = f"dp{dp}tp{a.tp}"
    out = {
        "metric": metric,
        "value": round(total_q / t_max, 4) if t_max > 0 else 0.0,
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
        "config": {"model": a.model, "global_batch": a.batch * dp, "seq_len": seq_max, "max_model_len": eng.runner.max_len,
                   "parallelism": par,
                   "prompt_tokens_mean": round(total_p / max(1.0, total_ans), 1),
                   "max_new_tokens": a.max_new_tokens, "path": a.path, "mode": a.mode,
                   "client": a.client if a.path != "engine" else None,
                   "server_timeouts": "production 15s/30s" if a.production else "bench 600s",
                   "weight_layout": "one (fragment-packed)" if getattr(eng.model, "_packed", False) else "row-major + decode copies",
                   "resident_weight_gb_per_rank": round(eng.model.resident_weight_bytes() / 1e9, 2)},
        "p50_latency_ms": round(p50, 2),
        "p99_latency_ms": _pct(lats, 0.99),
        "generated_tokens_per_s": round(total_gen / t_max, 1) if t_max > 0 else 0.0,
        "decode_steps": stats.get("decode_steps"),
        "prefill_steps": stats.get("prefill_steps"),
        "mixed_steps": stats.get("mixed_steps"),
        "dist": {"world_size": world, "tp": a.tp, "dp": dp, "devices": devices,
                 "backend": _backend(), "custom_allreduce": ps.custom_ar is not None,
                 "step_bus": type(eng.bus).__name__ if eng.bus is not None else None},
    }
    if a.mode != "wave" or a.production:  # rank-0 replica's request-level detail
        ttft = [r["ttft_ms"] for r in ok if r.get("ttft_ms") is not None]
        tpot = [(r["latency_ms"] - r["ttft_ms"]) / (r["completion_tokens"] - 1) for r in ok
                if r.get("ttft_ms") is not None and r.get("completion_tokens", 0) > 1]
        out["requests"] = {"sent": len(res) * dp, "ok_rank0": len(ok), "rejected_503_rank0":
                           sum(r.get("http_status") == 503 for r in res),
                           "timeout_504_rank0": sum(r.get("http_status") == 504 for r in res),
                           "deadline_truncated_rank0": sum(r.get("finish_reason") == "deadline" for r in ok),
                           "refused_cannot_finish_rank0": stats.get("infeasible_rejected"),
                           "value_counts": "complete answers (deadline-truncated excluded)"}
        out["tpot_model_ms"] = stats.get("tpot_model_ms")
        out["ttft_ms"] = {"p50": _pct(ttft, 0.5), "p99": _pct(ttft, 0.99)}
        out["tpot_ms"] = {"p50": _pct(tpot, 0.5), "p99": _pct(tpot, 0.99)}
        if a.mode == "poisson":
            out["config"]["rate_per_replica"] = a.rate
    line = json.dumps(out)
    print(line, flush=True)
    if a.out:
        with open(a.out, "w") as f:
            f.write(line + "\n")


def _backend():
    import torch.distributed as dist

    return dist.get_backend() if dist.is_available() and dist.is_initialized() else None


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
    for w in waves:
        # wave boundary: the previous wave's last decode step -> this wave's first arrival -> first prefill
        prev = [e[0] for e in dec if e[0] < w[0][0]]
        nxt = [e[0] for e in pre if e[0] >= w[0][0]]
        pls = [e for e in ev if e[1] == "plaunch" and e[0] >= w[0][0]]
        if prev and nxt:
            lt = f", first prefill launched +{(pls[0][0] - w[0][0]) * 1e3:.1f} ms ({pls[0][3]:.1f} ms host)" if pls else ""
            print(f"[trace] boundary: last decode -> first add {(w[0][0] - prev[-1]) * 1e3:.1f} ms, "
                  f"first add -> first prefill {(nxt[0] - w[0][0]) * 1e3:.1f} ms{lt}", file=sys.stderr)
            # where the boundary goes: answers resolved (detokenized) on the engine thread ->
            # first new request submitted by an HTTP handler -> added by the engine thread
            res = [e[0] for e in ev if e[1] == "resolved" and prev[-1] <= e[0] < w[0][0]]
            sub = [e[0] for e in ev if e[1] == "submit" and prev[-1] <= e[0] <= w[0][0]]
            if res and sub:
                print(f"[trace]   last decode -> answers resolved {(res[-1] - prev[-1]) * 1e3:.1f} ms, "
                      f"-> first submit {(sub[0] - res[-1]) * 1e3:.1f} ms, -> first add {(w[0][0] - sub[0]) * 1e3:.1f} ms",
                      file=sys.stderr)
        # arrival timeline of the wave: k-th request submitted (server side) and added (engine)
        sub_w = [e[0] for e in ev if e[1] == "submit" and w[0][0] - 0.5 <= e[0] <= w[-1][0]]
        if sub_w:
            t_s = sub_w[0]
            ks = [k for k in (1, 4, 8, 12, 16, 32, 64) if k <= len(w)]
            print("[trace]   k-th submit / add (ms after the first submit): " + " ".join(
                f"{k}:{(sub_w[min(k, len(sub_w)) - 1] - t_s) * 1e3:.1f}/{(w[k - 1][0] - t_s) * 1e3:.1f}" for k in ks),
                file=sys.stderr)
        gaps = sorted(b[0] - a_[0] for a_, b in zip(w, w[1:]))
        print(f"[trace] adds {len(w)} first +{(w[0][0] - t0) * 1e3:.1f} ms last +{(w[-1][0] - t0) * 1e3:.1f} ms"
              + (f" median gap {gaps[len(gaps) // 2] * 1e3:.2f} ms max gap {gaps[-1] * 1e3:.2f} ms" if gaps else ""),
              file=sys.stderr)
    for e in pre:
        print(f"[trace] prefill +{(e[0] - t0) * 1e3:.1f} ms seqs {e[2]} tokens {e[3]}", file=sys.stderr)
    if dec:
        print(f"[trace] decode steps {len(dec)} first +{(dec[0][0] - t0) * 1e3:.1f} last +{(dec[-1][0] - t0) * 1e3:.1f} ms",
              file=sys.stderr)
        # host side of the decode pipeline: launch-to-launch interval, host ms inside decode_launch,
        # and ms blocked on the previous step's tokens (near 0 = the host, not the GPU, sets the pace)
        iv = sorted((b[0] - a_[0]) * 1e3 for a_, b in zip(dec, dec[1:]) if b[0] - a_[0] < 0.05)
        la = sorted(e[3] for e in ev if e[1] == "dlaunch")
        wt = sorted(e[3] for e in ev if e[1] == "dwait")

        def q(v, f):
            return v[min(len(v) - 1, int(f * len(v)))] if v else float("nan")
        print(f"[trace] decode interval p50 {q(iv, .5):.3f} p90 {q(iv, .9):.3f} ms; launch p50 {q(la, .5):.3f} "
              f"p90 {q(la, .9):.3f} ms; wait p10 {q(wt, .1):.3f} p50 {q(wt, .5):.3f} ms", file=sys.stderr)
    pl = sorted(e[3] for e in ev if e[1] == "plaunch")
    if pl:
        print(f"[trace] prefill launch host ms p50 {pl[len(pl) // 2]:.2f} max {pl[-1]:.2f} ({len(pl)} steps)",
              file=sys.stderr)


def main(argv=None) -> None:
    argv = list(sys.argv[1:] if argv is None else argv)
    a = parse(argv)
    if a.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(spawn_ranks(a.gpus, argv))
    run_rank(a)
    _teardown()


def _teardown() -> None:
    """Orderly exit of a multi-rank run: every rank waits for every other at a barrier, then tears
    its process groups down - no rank's process exits (closing its sockets) while a peer's
    collective could still be talking to it."""
    import torch.distributed as dist

    if dist.is_available() and dist.is_initialized():
        from k8s_llm_monitor_amd.parallel.state import barrier_all, destroy

        barrier_all()
        destroy()


if __name__ == "__main__":
    main()
