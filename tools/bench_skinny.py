"""Decode projections of a Llama-3-8B layer on MI355X: hipBLASLt (+ the unfused elementwise
kernels it needs) versus gemm_skinny over fragment-packed weights, per decode batch size.

  qkv      F.linear                               vs skinny slabs (reduced later by rope_and_cache)
  o        F.linear + fused_add_rms_norm          vs skinny slabs + reduce_add_rms_norm
  gate_up  F.linear + silu_mul                    vs skinny SWIGLU epilogue
  down     F.linear + fused_add_rms_norm          vs skinny slabs + reduce_add_rms_norm

Every variant is timed as 32 calls captured in one hipGraph (no host launch gaps, as in the
engine's decode graph), rotating over > 512 MiB of weight copies so the weights stream from HBM
as they do in a 32-layer step, not from the 256 MiB MALL.

    python tools/bench_skinny.py [--ms 1,16,64] [--splits 2,4,8]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from k8s_llm_monitor_amd import ops  # noqa: E402


def timeit(fn, iters: int, per_graph: int = 32) -> float:
    for i in range(3):
        fn(i)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    st = torch.cuda.Stream()
    with torch.cuda.stream(st):
        with torch.cuda.graph(g, stream=st):
            for i in range(per_graph):
                fn(i)
    torch.cuda.synchronize()
    g.replay()
    torch.cuda.synchronize()
    reps = max(1, iters // per_graph)
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        g.replay()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / (reps * per_graph) * 1e3  # us


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=320)
    ap.add_argument("--ms", default="1,16,32,64")
    ap.add_argument("--splits", default="4,6,8")
    ap.add_argument("--ops", default="qkv,o,gate_up,down")
    a = ap.parse_args()
    dev = "cuda"
    d, F, nq, eps = 4096, 14336, 6144, 1e-5
    shapes = {"qkv": (nq, d), "o": (d, d), "gate_up": (2 * F, d), "down": (d, F)}
    nw = torch.ones(d, device=dev, dtype=torch.bfloat16)
    for name in a.ops.split(","):
        N, K = shapes[name]
        ncopy = max(2, (512 << 20) // (N * K * 2) + 1)
        ws = [torch.randn(N, K, device=dev, dtype=torch.bfloat16) * 0.02 for _ in range(ncopy)]
        wps = [ops.pack_skinny(ops.interleave_gate_up(w) if name == "gate_up" else w) for w in ws]
        gb = N * K * 2 / 1e9
        for M in map(int, a.ms.split(",")):
            x = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
            xp = ops.pack_activation(x)
            r = torch.randn(M, d, device=dev, dtype=torch.bfloat16)
            y = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
            ob = torch.empty(M, d, device=dev, dtype=torch.bfloat16)
            act = torch.empty(M, F, device=dev, dtype=torch.bfloat16)

            def rep(impl, t):
                print(json.dumps({"op": name, "M": M, "impl": impl, "us": round(t, 2),
                                  "TBps": round(gb / t * 1e3, 2)}), flush=True)

            def base(i):
                torch.matmul(x, ws[i % ncopy].t(), out=y)
                if name == "gate_up":
                    ops.silu_mul(y, out=act)
                elif name in ("o", "down"):
                    ops.fused_add_rms_norm(y, r, nw, eps, out=ob)

            rep("hipblaslt" + ("+silu_mul" if name == "gate_up" else "+norm" if name in ("o", "down") else ""),
                timeit(base, a.iters))
            if name == "gate_up":
                rep("skinny swiglu", timeit(lambda i: ops.skinny_swiglu(x, wps[i % ncopy], out=act), a.iters))
                rep("skinny swiglu packedA",
                    timeit(lambda i: ops.skinny_swiglu(xp, wps[i % ncopy], out=act, rows=M), a.iters))
                continue
            if name == "qkv":
                for nt_tiles in (2, 4):
                    rep(f"skinny bf16 1slice nt{nt_tiles} packedA",
                        timeit(lambda i: ops.skinny_linear(xp, wps[i % ncopy], out=y, nt_tiles=nt_tiles, rows=M),
                               a.iters))
            wsp = ops.skinny_workspace(M, N, 16, dev)
            if name == "qkv":
                fn = lambda i, wsp=wsp: ops.skinny_slabs(xp, wps[i % ncopy], wsp, 0, rows=M)  # noqa: E731
            else:
                fn = lambda i, wsp=wsp: ops.proj_add_rms_norm(  # noqa: E731
                    xp, wps[i % ncopy], r, nw, eps, workspace=wsp, splits=0, out=ob, rows=M)
            rep("skinny auto packedA", timeit(fn, a.iters))
            for s in map(int, a.splits.split(",")):
                wsp = ops.skinny_workspace(M, N, s, dev)
                for tag, xa in (("", x), (" packedA", xp)):
                    if name == "qkv":
                        fn = lambda i, s=s, wsp=wsp, xa=xa: ops.skinny_slabs(xa, wps[i % ncopy], wsp, s,  # noqa: E731
                                                                             rows=M)
                    else:
                        fn = lambda i, s=s, wsp=wsp, xa=xa: ops.proj_add_rms_norm(  # noqa: E731
                            xa, wps[i % ncopy], r, nw, eps, workspace=wsp, splits=s, out=ob, rows=M)
                    rep(f"skinny s{s}{tag}", timeit(fn, a.iters))
        del ws, wps
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
