"""Latency vs message size of the IPC collectives (ops/csrc/custom_ar.hip), W processes sharing
ONE GPU (the only multi-rank setup the one-GPU pool allows; VERDICT r2 "do this" #3).

    python tools/bench_custom_ar.py [--world 2] [--iters 200] [--out profiles/r03/custom_ar_latency.jsonl]

Per size (8 KiB .. 16 MiB bf16) and per call kind - one-shot all-reduce (algo 0), two-shot (algo 1),
all-gather, all-to-all, and the fused row-parallel tail (rows x 4096 / 8192, 4 split-K slabs) -
ITERS calls are captured in one hipGraph and replayed; the replay is timed with events and the
max over ranks is reported.  Two processes on one GPU share its CUs and HBM, and their "peer"
reads are local HBM reads, not xGMI: the numbers bound the protocol's fixed cost (launch, flag
round trips, fences), NOT the 8-GPU xGMI bandwidth - no 1 -> 8 GPU curve exists until the driver's
8-GPU node runs the scaling bench.
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

SIZES_KIB = [8, 32, 128, 512, 1024, 2048, 4096, 8192, 16384]


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _time_graph(torch, fn, iters: int) -> float:
    """Mean us per call of `fn` over `iters` calls captured in one graph."""
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        fn()
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(iters):
            fn()
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    best = float("inf")
    for _ in range(3):
        e0.record()
        g.replay()
        e1.record()
        torch.cuda.synchronize()
        best = min(best, e0.elapsed_time(e1) * 1e3 / iters)
    return best


def _rank(rank: int, world: int, port: int, iters: int, q) -> None:
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    import torch
    import torch.distributed as dist

    from k8s_llm_monitor_amd.parallel.custom_ar import CustomAllReduce

    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.cuda.set_device(0)
    car = CustomAllReduce(rank, world, max_bytes=32 << 20)
    dev = torch.device("cuda:0")
    rows = []

    def agree(us: float) -> float:
        t = torch.tensor([us], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item())

    for kib in SIZES_KIB:
        n = kib * 1024 // 2
        x = torch.randn(n, device=dev).to(torch.bfloat16)
        row = {"bytes": kib * 1024, "world": world}
        for name, fn in (("one_shot", lambda: car.all_reduce_(x, 0)), ("two_shot", lambda: car.all_reduce_(x, 1))):
            dist.barrier()
            row[name + "_us"] = round(agree(_time_graph(torch, fn, iters)), 2)
        g_in = x[: n // world].contiguous()
        dist.barrier()
        row["all_gather_us"] = round(agree(_time_graph(torch, lambda: car.all_gather(g_in), iters)), 2)
        a_in = x.view(world, -1)
        dist.barrier()
        row["all_to_all_us"] = round(agree(_time_graph(torch, lambda: car.all_to_all(a_in), iters)), 2)
        rows.append(row)
    # fused tail: slab sum + all-reduce + residual + RMSNorm + packed write for decode rows
    for d in (4096, 8192):
        for M in (1, 16, 64):
            ns = 4
            slabs = torch.randn(ns, M, d, device=dev)
            res = torch.randn(M, d, device=dev).to(torch.bfloat16)
            w = torch.ones(d, device=dev, dtype=torch.bfloat16)
            out = torch.empty(-(-M // 16) * 16 * d, device=dev, dtype=torch.bfloat16)
            dist.barrier()
            us = agree(_time_graph(torch, lambda: car.fused_tail(slabs, ns, res, w, 1e-5, out, True), iters))
            rows.append({"kind": "fused_tail", "M": M, "d": d, "slabs": ns, "world": world, "us": round(us, 2)})
    err = car.error()
    car.close()
    dist.destroy_process_group()
    q.put((rank, rows, err))


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--world", type=int, default=2)
    ap.add_argument("--iters", type=int, default=200)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    import multiprocessing as mp

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank, args=(r, a.world, port, a.iters, q), daemon=True) for r in range(a.world)]
    for p in procs:
        p.start()
    got = {}
    for _ in procs:
        r, rows, err = q.get(timeout=600)
        got[r] = (rows, err)
    for p in procs:
        p.join(timeout=30)
    rows, err = got[0]
    if any(e for _, e in got.values()):
        print("ERROR: a collective timed out", file=sys.stderr)
        sys.exit(1)
    lines = [json.dumps(r) for r in rows]
    print("\n".join(lines))
    if a.out:
        with open(a.out, "w") as f:
            f.write("\n".join(lines) + "\n")


if __name__ == "__main__":
    main()
