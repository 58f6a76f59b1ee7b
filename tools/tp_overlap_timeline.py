#!/usr/bin/env python
"""TP prefill communication/computation overlap on ONE GPU.

Two (or more) TP ranks share cuda:0 - the pool has one-GPU boxes, so this is a timeline of the
mechanism, not an xGMI measurement.  Every rank builds the same Llama-shaped model sharded TP ways
and runs one prefill step of ``--seqs`` x ``--len`` tokens two ways:

* serial     - every row-parallel all-reduce on the compute stream (``tp_all_reduce``);
* overlapped - two micro-batches of whole sequences, every all-reduce queued asynchronously
  (``tp_all_reduce_async``: the IPC all-reduce on the high-priority comm stream) while the other
  micro-batch's GEMMs / attention run on the compute stream (``CausalLM._prefill_overlap``).

It prints one JSON line per rank (ms per step of each form, max |overlapped - serial| of the
logits) and, with ``--prof DIR``, each rank runs under its own ``rocprofv3 --kernel-trace`` so that
``--analyze DIR`` can report, from the per-rank databases, how much of the all-reduce kernels'
time ran concurrently with compute kernels of the same rank and on which streams.

    python tools/tp_overlap_timeline.py --world 2 [--model llama-3-8b --layers 8 --seqs 4 --len 512]
    python tools/tp_overlap_timeline.py --world 2 --prof gpurun_out/ovl   # per-rank kernel traces
    python tools/tp_overlap_timeline.py --analyze gpurun_out/ovl
"""
from __future__ import annotations

import argparse
import glob
import json
import os
import sqlite3
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def rank_main(a) -> None:
    import numpy as np
    import torch
    import torch.distributed as dist

    from k8s_llm_monitor_amd.engine.runner import ModelRunner
    from k8s_llm_monitor_amd.models import AttnMeta, CausalLM, get_config
    from k8s_llm_monitor_amd.parallel.state import destroy, init_parallel

    ps = init_parallel(tp_size=a.world)
    dev = ps.device
    cfg = get_config(a.model)
    if a.layers:
        cfg = cfg.replace(n_layers=a.layers)
    m = CausalLM(cfg, device=dev, dtype=torch.bfloat16, seed=3, pstate=ps)
    lens = [a.len] * a.seqs
    cu = np.concatenate([[0], np.cumsum(lens)]).astype(np.int32)
    T = int(cu[-1])
    g = torch.Generator().manual_seed(11)
    ids = torch.randint(0, cfg.vocab_size, (T,), generator=g, dtype=torch.int32).to(dev)
    pos = torch.cat([torch.arange(n, dtype=torch.int32) for n in lens]).to(dev)

    from k8s_llm_monitor_amd import ops

    def meta_for(c, p):
        # the q-block schedule on the device, as the engine's runner stages it (no per-call host copy)
        qs, st = ops.prefill_qblocks([int(v) for v in c])
        return AttnMeta(is_prefill=True, positions=p,
                        slot_mapping=torch.full((len(p),), -1, dtype=torch.int32, device=dev),
                        cu_seqlens=torch.tensor(c, dtype=torch.int32, device=dev),
                        qb_seq=torch.tensor(qs, dtype=torch.int32, device=dev),
                        qb_start=torch.tensor(st, dtype=torch.int32, device=dev),
                        logits_idx=torch.tensor(np.asarray(c[1:]) - 1, dtype=torch.int64, device=dev))

    kA = ModelRunner._micro_split(cu, 0, min_rows=0)
    TA = int(cu[kA])
    serial_meta = meta_for(cu, pos)
    over_meta = meta_for(cu, pos)
    over_meta.micro = (meta_for(cu[: kA + 1], pos[:TA]), meta_for(cu[kA:] - cu[kA], pos[TA:]), TA)
    car = ps.custom_ar
    fits = car is not None and car.fits(torch.empty(TA, cfg.d_model, dtype=torch.bfloat16, device=dev))

    def step(meta):
        with torch.no_grad():
            return m.forward(ids, meta, None)

    def sync():
        if dev.type == "cuda":
            torch.cuda.synchronize(dev)

    def timed(meta, n):
        dist.barrier(group=ps.cpu_group)
        sync()
        t0 = time.perf_counter()
        for _ in range(n):
            out = step(meta)
        sync()
        return (time.perf_counter() - t0) * 1e3 / n, out

    for _ in range(a.warmup):
        step(serial_meta)
        step(over_meta)
    res = {"serial": [], "overlapped": []}
    for _ in range(a.rounds):  # interleaved A/B
        t, ser = timed(serial_meta, a.iters)
        res["serial"].append(t)
        t, ovl = timed(over_meta, a.iters)
        res["overlapped"].append(t)
    err = (ovl.float() - ser.float()).abs().max().item()
    rec = {"rank": ps.rank, "world": a.world, "model": cfg.name, "layers": cfg.n_layers, "tokens": T,
           "micro_rows": [TA, T - TA], "ipc_all_reduce": bool(fits),
           "ms_serial": round(min(res["serial"]), 3), "ms_overlapped": round(min(res["overlapped"]), 3),
           "ms_serial_all": [round(x, 3) for x in res["serial"]],
           "ms_overlapped_all": [round(x, 3) for x in res["overlapped"]],
           "bitwise_equal": bool(torch.equal(ovl, ser)), "max_abs_diff": err}
    print(json.dumps(rec), flush=True)
    dist.barrier(group=ps.cpu_group)
    destroy()


def launch(a) -> int:
    import socket

    # the launcher never touches the GPU; every rank is a fresh child process (under its own
    # rocprofv3 with --prof)
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    procs = []
    for r in range(a.world):
        env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(r), LOCAL_RANK=str(r),
                   WORLD_SIZE=str(a.world), K8SLLM_DEVICE=a.device, K8SLLM_DIST_BACKEND="gloo")
        cmd = [sys.executable, os.path.abspath(__file__), "--rank", str(r)] + a.passthru
        if a.prof:
            d = os.path.join(a.prof, f"rank{r}")
            cmd = ["rocprofv3", "--kernel-trace", "-d", d, "-o", "run", "--"] + cmd
        procs.append(subprocess.Popen(cmd, env=env))
    rc = 0
    for p in procs:
        rc = rc or p.wait()
    return rc


def _intervals_overlap(a0, a1, spans) -> int:
    """ns of [a0, a1) covered by the union of ``spans`` (sorted, possibly overlapping)."""
    cov, cur0, cur1 = 0, None, None
    for s0, s1 in spans:
        s0, s1 = max(s0, a0), min(s1, a1)
        if s1 <= s0:
            continue
        if cur1 is None or s0 > cur1:
            if cur1 is not None:
                cov += cur1 - cur0
            cur0, cur1 = s0, s1
        else:
            cur1 = max(cur1, s1)
    if cur1 is not None:
        cov += cur1 - cur0
    return cov


def analyze(d: str) -> None:
    """Per rank: the all-reduce kernels (``car_kernel``) of the overlapped steps and how much of
    their time ran beside the rank's compute kernels, plus the streams each group used."""
    for db in sorted(glob.glob(os.path.join(d, "rank*", "**", "*results.db"), recursive=True)):
        c = sqlite3.connect(db)
        cols = [r[1] for r in c.execute("pragma table_info(kernels)")]
        sid = "stream_id" if "stream_id" in cols else ("queue_id" if "queue_id" in cols else None)
        q = f"select name, start, end{', ' + sid if sid else ''} from kernels order by start"
        rows = c.execute(q).fetchall()
        ar = [r for r in rows if "car_kernel" in r[0]]
        comp = [r for r in rows if "car_" not in r[0]]
        spans = sorted((r[1], r[2]) for r in comp)
        tot = sum(r[2] - r[1] for r in ar)
        cov = sum(_intervals_overlap(r[1], r[2], spans) for r in ar)
        streams_ar = sorted({r[3] for r in ar}) if sid else []
        streams_comp = sorted({r[3] for r in comp}) if sid else []
        # the overlapped form's all-reduces run on a stream of their own: split by stream
        by_stream = {}
        for r in ar:
            k = r[3] if sid else 0
            n, t, cv = by_stream.get(k, (0, 0, 0))
            by_stream[k] = (n + 1, t + r[2] - r[1], cv + _intervals_overlap(r[1], r[2], spans))
        print(json.dumps({
            "db": os.path.relpath(db, d), "stream_column": sid, "ar_kernels": len(ar),
            "ar_time_ms": round(tot / 1e6, 3), "ar_time_beside_compute_ms": round(cov / 1e6, 3),
            "ar_streams": streams_ar, "compute_streams": streams_comp,
            "per_ar_stream": {str(k): {"kernels": v[0], "ms": round(v[1] / 1e6, 3),
                                       "beside_compute_ms": round(v[2] / 1e6, 3),
                                       "overlap_frac": round(v[2] / max(v[1], 1), 3)}
                              for k, v in by_stream.items()}}))


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--world", type=int, default=2)
    ap.add_argument("--rank", type=int, default=-1, help="internal: run one rank")
    ap.add_argument("--model", default="llama-3-8b")
    ap.add_argument("--layers", type=int, default=8)
    ap.add_argument("--seqs", type=int, default=4)
    ap.add_argument("--len", type=int, default=512)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--iters", type=int, default=3)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--device", default="cuda:0", help="every rank's device (cpu: a plumbing check)")
    ap.add_argument("--prof", default="")
    ap.add_argument("--analyze", default="")
    a = ap.parse_args()
    if a.analyze:
        analyze(a.analyze)
        return
    if a.rank >= 0:
        rank_main(a)
        return
    a.passthru = ["--world", str(a.world), "--model", a.model, "--layers", str(a.layers), "--seqs", str(a.seqs),
                  "--len", str(a.len), "--warmup", str(a.warmup), "--iters", str(a.iters), "--rounds", str(a.rounds)]
    sys.exit(launch(a))


if __name__ == "__main__":
    main()
