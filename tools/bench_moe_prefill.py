"""Mixtral-8x7B MoE prefill MLP on MI355X: the grouped expert GEMMs (ops/csrc/moe_gemm.hip, one
launch per projection, device offsets, no host sync) versus the per-expert hipBLASLt loop (host
sync on the offsets).  T tokens x top-2 over 8 experts, d 4096, F 14336.

    python tools/bench_moe_prefill.py [--tokens 16384]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from k8s_llm_monitor_amd import ops  # noqa: E402


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--tokens", type=int, default=16384)
    ap.add_argument("--iters", type=int, default=5)
    a = ap.parse_args()
    dev = "cuda"
    E, d, F, K = 8, 4096, 14336, 2
    T = a.tokens
    torch.manual_seed(0)
    x = torch.randn(T, d, device=dev, dtype=torch.bfloat16)
    logits = torch.randn(T, E, device=dev)
    ids, w = ops.moe_route(logits, K, True)
    w13 = (torch.randn(E, 2 * F, d, device=dev, dtype=torch.bfloat16) * 0.02)
    w13 = torch.stack([ops.interleave_gate_up(we) for we in w13]).contiguous()
    w2 = (torch.randn(E, d, F, device=dev, dtype=torch.bfloat16) * 0.02)

    def grouped():
        offsets, sorted_idx, inv_idx = ops.moe_align(ids, E)
        xs = ops.gather_rows(x, sorted_idx, K)
        h = ops.moe_grouped_gemm(xs, w13, offsets, swiglu=True, zero_fill=False)
        ys = ops.moe_grouped_gemm(h, w2, offsets, zero_fill=False)
        return ops.moe_combine(ys, inv_idx, w, T)

    def loop():
        offsets, sorted_idx, inv_idx = ops.moe_align(ids, E)
        xs = ops.gather_rows(x, sorted_idx, K)
        ys = torch.empty_like(xs)
        off = offsets.tolist()
        for e in range(E):
            lo, hi = off[e], off[e + 1]
            if hi > lo:
                h = ops.silu_mul(torch.nn.functional.linear(xs[lo:hi], w13[e]), interleaved=True)
                ys[lo:hi] = torch.nn.functional.linear(h, w2[e])
        return ops.moe_combine(ys, inv_idx, w, T)

    ya, yb = grouped(), loop()
    err = float((ya.float() - yb.float()).abs().max())
    flops = 2 * T * K * (d * 2 * F + F * d)
    res = {"tokens": T, "max_abs_diff": round(err, 4)}
    for _ in range(2):
        for name, fn in (("grouped", grouped), ("loop", loop)):
            for _ in range(2):
                fn()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(a.iters):
                fn()
            torch.cuda.synchronize()
            dt = (time.perf_counter() - t0) / a.iters
            res[name + "_ms"] = min(res.get(name + "_ms", 1e9), round(dt * 1e3, 3))
    for name in ("grouped", "loop"):
        res[name + "_PFps"] = round(flops / (res[name + "_ms"] * 1e-3) / 1e15, 3)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
