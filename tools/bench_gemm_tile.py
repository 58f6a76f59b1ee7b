"""Prefill GEMMs on MI355X: the 256 x 256 MFMA tile kernel (w4: one barrier per k-tile, w4s: two) (ops/csrc/gemm_tile.hip) against
hipBLASLt (torch F.linear), at the Llama-3-8B prefill-chunk shapes (16384 tokens) and the
Mixtral-8x7B grouped expert shapes (top-2 of 8).  Random operands, interleaved rounds, hipGraph
replay of back-to-back calls; the SwiGLU rows compare the fused epilogue with F.linear + silu_mul.

    python tools/bench_gemm_tile.py [--tokens 16384] [--rounds 3]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from k8s_llm_monitor_amd import ops  # noqa: E402
from tools.bench_skinny import timeit  # noqa: E402

F_ = torch.nn.functional


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--tokens", type=int, default=16384)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--iters", type=int, default=16)
    ap.add_argument("--only", default="")
    ap.add_argument("--impl", default="", help="comma list of implementations to time (default all)")
    a = ap.parse_args()
    dev = "cuda"
    T = a.tokens
    torch.manual_seed(0)
    cases = []
    d, F = 4096, 14336
    x = torch.randn(T, d, device=dev, dtype=torch.bfloat16)
    xf = torch.randn(T, F, device=dev, dtype=torch.bfloat16)
    for name, N, K in (("qkv", 6144, d), ("o", d, d), ("down", d, F)):
        w = torch.randn(N, K, device=dev, dtype=torch.bfloat16) * 0.02
        xin = xf if K == F else x
        y = torch.empty(T, N, device=dev, dtype=torch.bfloat16)
        cases.append((name, 2 * T * N * K, {
            "w4": (lambda i, xin=xin, w=w, y=y: ops.gemm_tile(xin, w, out=y, algo=0)),
            "w4s": (lambda i, xin=xin, w=w, y=y: ops.gemm_tile(xin, w, out=y, algo=1)),
            "hipblaslt": (lambda i, xin=xin, w=w, y=y: torch.matmul(xin, w.t(), out=y)),
        }))
    # qkv + RoPE + paged-cache write, as the prefill layer runs it: tile GEMM with the RoPE epilogue
    # + cache-only pass, vs hipBLASLt + the rotate-and-cache pass
    from k8s_llm_monitor_amd.ops import reference as ref
    wq = torch.randn(6144, d, device=dev, dtype=torch.bfloat16) * 0.02
    yq = torch.empty(T, 6144, device=dev, dtype=torch.bfloat16)
    cs = ref.rope_cos_sin(max(T, 8192), 128, 500000.0).to(dev).float().contiguous()
    pos = (torch.arange(T, device=dev) % 8192).to(torch.int32)
    nb = (T + 15) // 16
    kc = torch.empty(nb, 8, 16, 16, 8, device=dev, dtype=torch.bfloat16)
    vc = torch.empty(nb, 8, 128, 16, device=dev, dtype=torch.bfloat16)
    slots = torch.arange(T, device=dev, dtype=torch.int32)
    cases.append(("qkv+rope+cache", 2 * T * 6144 * d, {
        "w4s": (lambda i: ops.rope_and_cache(ops.gemm_tile(x, wq, out=yq, algo=1, rope=(pos, cs, 40)), pos, cs,
                                             kc, vc, slots, 32, 8, 128, apply_rope=False)),
        "hipblaslt": (lambda i: ops.rope_and_cache(torch.matmul(x, wq.t(), out=yq), pos, cs, kc, vc, slots,
                                                   32, 8, 128, apply_rope=True)),
        "w4s_gemm_only": (lambda i: ops.gemm_tile(x, wq, out=yq, algo=1, rope=(pos, cs, 40))),
        "rope_cache_only": (lambda i: ops.rope_and_cache(yq, pos, cs, kc, vc, slots, 32, 8, 128, apply_rope=True)),
        "cache_only": (lambda i: ops.rope_and_cache(yq, pos, cs, kc, vc, slots, 32, 8, 128, apply_rope=False)),
    }))
    # the fused-norm epilogues vs their plain forms, same operands: gate_up + SwiGLU with / without
    # the row scale, qkv + RoPE with / without it, o with the residual epilogue vs plain
    ssq = (torch.rand(T, d // 128, device=dev) * 128 + 64).contiguous()
    resid = torch.randn(T, d, device=dev, dtype=torch.bfloat16)
    hwb = torch.empty(T, d, device=dev, dtype=torch.bfloat16)
    ssb = torch.empty(T, d // 128, device=dev, dtype=torch.float32)
    nwv = torch.ones(d, device=dev, dtype=torch.bfloat16)
    wo_ = torch.randn(d, d, device=dev, dtype=torch.bfloat16) * 0.02
    yo = torch.empty(T, d, device=dev, dtype=torch.bfloat16)
    cases.append(("qkv+rope_rs", 2 * T * 6144 * d, {
        "plain": (lambda i: ops.gemm_tile(x, wq, out=yq, algo=1, rope=(pos, cs, 40))),
        "rowscale": (lambda i: ops.gemm_tile(x, wq, out=yq, algo=1, rope=(pos, cs, 40), rowscale=(ssq, 1e-5))),
    }))
    cases.append(("o_resid", 2 * T * d * d, {
        "plain": (lambda i: ops.gemm_tile(x, wo_, out=yo, algo=1)),
        "resid": (lambda i: ops.gemm_tile_resid(x, wo_, resid, nwv, hw=hwb, ss=ssb)),
    }))
    w13 = ops.interleave_gate_up(torch.randn(2 * F, d, device=dev, dtype=torch.bfloat16) * 0.02).contiguous()
    gu = torch.empty(T, 2 * F, device=dev, dtype=torch.bfloat16)
    act = torch.empty(T, F, device=dev, dtype=torch.bfloat16)
    cases.append(("gate_up+swiglu_rs", 2 * T * 2 * F * d, {
        "plain": (lambda i: ops.gemm_tile(x, w13, swiglu=True, out=act, algo=1)),
        "rowscale": (lambda i: ops.gemm_tile(x, w13, swiglu=True, out=act, algo=1, rowscale=(ssq, 1e-5))),
    }))
    cases.append(("gate_up+swiglu", 2 * T * 2 * F * d, {
        "w4": (lambda i: ops.gemm_tile(x, w13, swiglu=True, out=act, algo=0)),
        "w4s": (lambda i: ops.gemm_tile(x, w13, swiglu=True, out=act, algo=1)),
        "hipblaslt": (lambda i: ops.silu_mul(torch.matmul(x, w13.t(), out=gu), out=act, interleaved=True)),
        "hipblaslt_gemm_only": (lambda i: torch.matmul(x, w13.t(), out=gu)),
    }))
    # Mixtral grouped experts: T tokens x top-2 over 8 experts (balanced-ish random routing)
    E = 8
    ids, _ = ops.moe_route(torch.randn(T, E, device=dev), 2, True)
    offsets, _, _ = ops.moe_align(ids, E)
    rows = 2 * T
    off = offsets.tolist()
    xs = torch.randn(rows, d, device=dev, dtype=torch.bfloat16)
    hs = torch.randn(rows, F, device=dev, dtype=torch.bfloat16)
    we13 = torch.stack([ops.interleave_gate_up(torch.randn(2 * F, d, device=dev, dtype=torch.bfloat16) * 0.02)
                        for _ in range(E)]).contiguous()
    we2 = torch.randn(E, d, F, device=dev, dtype=torch.bfloat16) * 0.02
    ha = torch.empty(rows, F, device=dev, dtype=torch.bfloat16)
    ys = torch.empty(rows, d, device=dev, dtype=torch.bfloat16)

    def loop13(i):
        for e in range(E):
            lo, hi = off[e], off[e + 1]
            if hi > lo:
                ops.silu_mul(F_.linear(xs[lo:hi], we13[e]), out=ha[lo:hi], interleaved=True)

    def loop2(i):
        for e in range(E):
            lo, hi = off[e], off[e + 1]
            if hi > lo:
                torch.matmul(hs[lo:hi], we2[e].t(), out=ys[lo:hi])

    cases.append(("moe_w13+swiglu", 2 * rows * 2 * F * d, {
        "w4": (lambda i: ops.gemm_tile(xs, we13, offsets, swiglu=True, out=ha, algo=0)),
        "w4s": (lambda i: ops.gemm_tile(xs, we13, offsets, swiglu=True, out=ha, algo=1)),
        "moe_gemm128": (lambda i: ops.moe_grouped_gemm(xs, we13, offsets, swiglu=True, out=ha)),
        "hipblaslt_loop": loop13,
    }))
    cases.append(("moe_w2", 2 * rows * d * F, {
        "w4": (lambda i: ops.gemm_tile(hs, we2, offsets, out=ys, algo=0)),
        "w4s": (lambda i: ops.gemm_tile(hs, we2, offsets, out=ys, algo=1)),
        "moe_gemm128": (lambda i: ops.moe_grouped_gemm(hs, we2, offsets, out=ys)),
        "hipblaslt_loop": loop2,
    }))
    for name, flops, impls in cases:
        if a.only and name not in a.only.split(","):
            continue
        res: dict = {}
        for _ in range(a.rounds):
            for tag, fn in impls.items():
                if a.impl and tag not in a.impl.split(","):
                    continue
                res.setdefault(tag, []).append(timeit(fn, a.iters, per_graph=4))
        for tag, ts in res.items():
            t = min(ts)
            print(json.dumps({"op": name, "tokens": T, "impl": tag, "us": round(t, 1),
                              "us_all": [round(v, 1) for v in ts], "PFps": round(flops / t / 1e9, 3)}), flush=True)


if __name__ == "__main__":
    main()
