#!/usr/bin/env python
"""What the fused prefill epilogues cost the 256 x 256 tile GEMM: the Llama-3-8B qkv projection
(16384 x 6144 x 4096) plain, with the RoPE epilogue, and with RoPE + the deferred-norm row scale
(the engine's form); the o projection plain vs the residual/norm epilogue.  Interleaved rounds,
hipGraph replay of back-to-back calls (tools/bench_skinny.timeit).

    python tools/bench_tile_epilogues.py [--tokens 16384 --rounds 3]"""
from __future__ import annotations

import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from k8s_llm_monitor_amd import ops  # noqa: E402
from tools.bench_skinny import timeit  # noqa: E402


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--tokens", type=int, default=16384)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--iters", type=int, default=16)
    a = ap.parse_args()
    dev, T, d = "cuda", a.tokens, 4096
    torch.manual_seed(0)
    x = torch.randn(T, d, device=dev, dtype=torch.bfloat16)
    wq = torch.randn(6144, d, device=dev, dtype=torch.bfloat16) * 0.02
    wo = torch.randn(d, d, device=dev, dtype=torch.bfloat16) * 0.02
    pos = (torch.arange(T, device=dev, dtype=torch.int32) % 1700)
    cs = torch.randn(8192, 128, device=dev, dtype=torch.float32)
    ssp = torch.rand(T, d // 128, device=dev, dtype=torch.float32) + 0.5
    out_q = torch.empty(T, 6144, device=dev, dtype=torch.bfloat16)
    resid = torch.randn(T, d, device=dev, dtype=torch.bfloat16)
    nw = torch.ones(d, device=dev, dtype=torch.bfloat16)
    hw = torch.empty_like(resid)
    ss = torch.empty(T, d // 128, device=dev, dtype=torch.float32)
    w13p = ops.pack_skinny(ops.interleave_gate_up8(torch.randn(28672, d, device=dev, dtype=torch.bfloat16) * 0.02))
    out_gu = torch.empty(T, 14336, device=dev, dtype=torch.bfloat16)
    cases = {
        "qkv_plain": (lambda _i: ops.gemm_tile(x, wq, out=out_q, algo=ops.TILE_ALGO), 2 * T * 6144 * d),
        "qkv_rope": (lambda _i: ops.gemm_tile(x, wq, out=out_q, rope=(pos, cs, 40), algo=ops.TILE_ALGO), 2 * T * 6144 * d),
        "qkv_rope_rs": (lambda _i: ops.gemm_tile(x, wq, out=out_q, rope=(pos, cs, 40), rowscale=(ssp, 1e-5), algo=ops.TILE_ALGO),
                        2 * T * 6144 * d),
        "o_plain": (lambda _i: ops.gemm_tile(x, wo, out=hw, algo=ops.TILE_ALGO), 2 * T * d * d),
        "o_resid": (lambda _i: ops.gemm_tile_resid(x, wo, resid, nw, hw, ss), 2 * T * d * d),
        # the engine's gate_up: packed W (one layout), SwiGLU over the per-16 pairing, row-scaled
        "gu_swiglu8_rs": (lambda _i: ops.gemm_tile(x, w13p, swiglu=8, out=out_gu, rowscale=(ssp, 1e-5),
                                                   algo=ops.TILE_ALGO), 2 * T * 28672 * d),
    }
    res: dict = {k: [] for k in cases}
    for _ in range(a.rounds):
        for k, (fn, flop) in cases.items():
            us = timeit(fn, a.iters)
            res[k].append(us)
    for k, (fn, flop) in cases.items():
        us = sorted(res[k])[len(res[k]) // 2]
        print(json.dumps({"case": k, "tokens": T, "us": round(us, 1), "pflops": round(flop / us / 1e9, 3),
                          "all_us": [round(u, 1) for u in res[k]]}), flush=True)


if __name__ == "__main__":
    main()
