"""Where the prefill tile GEMM loses to hipBLASLt: time both at one (M, N) over a sweep of K and fit
t = fixed + per_k * K.  `fixed` is the per-launch + per-tile prologue / epilogue cost (the tile's
first DMA burst, the store tail), `per_k` the main loop.  Random operands, hipGraph replay.

    python tools/gemm_k_sweep.py [--m 16384] [--n 4096] [--ks 512,1024,2048,4096,8192]
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


def fit(ks: list[int], ts: list[float]) -> tuple[float, float]:
    n = len(ks)
    mk, mt = sum(ks) / n, sum(ts) / n
    b = sum((k - mk) * (t - mt) for k, t in zip(ks, ts)) / sum((k - mk) ** 2 for k in ks)
    return mt - b * mk, b


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--m", type=int, default=16384)
    ap.add_argument("--n", type=int, default=4096)
    ap.add_argument("--ks", default="512,1024,2048,4096,8192")
    ap.add_argument("--iters", type=int, default=16)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--algos", default="1")
    ap.add_argument("--no-blas", action="store_true")
    ap.add_argument("--packed", action="store_true", help="also time the fragment-packed weight layout")
    a = ap.parse_args()
    torch.manual_seed(0)
    ks = [int(k) for k in a.ks.split(",")]
    impls: dict = {}
    for K in ks:
        x = torch.randn(a.m, K, device="cuda", dtype=torch.bfloat16)
        w = torch.randn(a.n, K, device="cuda", dtype=torch.bfloat16) * 0.02
        y = torch.empty(a.m, a.n, device="cuda", dtype=torch.bfloat16)
        for al in a.algos.split(","):
            impls.setdefault(f"tile{al}", {})[K] = lambda i, x=x, w=w, y=y, al=int(al): ops.gemm_tile(x, w, out=y, algo=al)
        if a.packed:  # the same GEMM over the decode GEMMs' fragment-packed weight layout
            wp = ops.pack_skinny(w)
            al = int(a.algos.split(",")[0])
            if not torch.equal(ops.gemm_tile(x, wp, algo=al), ops.gemm_tile(x, w, algo=al)):
                raise SystemExit(f"packed W differs from row-major W at K={K}")
            impls.setdefault(f"tile{al}_packed", {})[K] = lambda i, x=x, wp=wp, y=y, al=al: ops.gemm_tile(x, wp, out=y, algo=al)
        if not a.no_blas:
            impls.setdefault("hipblaslt", {})[K] = lambda i, x=x, w=w, y=y: torch.matmul(x, w.t(), out=y)
        if "," in a.algos:  # every schedule must give the same bits (same MFMA order per accumulator)
            outs = [ops.gemm_tile(x, w, algo=int(al)) for al in a.algos.split(",")]
            for al, o in zip(a.algos.split(","), outs):
                if not torch.equal(o, outs[0]):
                    raise SystemExit(f"algo {al} differs from algo {a.algos.split(',')[0]} at K={K}")
    res: dict = {}
    for _ in range(a.rounds):
        for tag, by_k in impls.items():
            for K, fn in by_k.items():
                res.setdefault((tag, K), []).append(timeit(fn, a.iters, per_graph=4))
    for tag in impls:
        ts = [min(res[(tag, K)]) for K in ks]
        if len(ks) < 2:
            print(json.dumps({"impl": tag, "M": a.m, "N": a.n, "K": ks[0], "us": round(ts[0], 1),
                              "us_all": [round(v, 1) for v in res[(tag, ks[0])]],
                              "PFps": round(2 * a.m * a.n * ks[0] / ts[0] / 1e9, 3)}), flush=True)
            continue
        f, b = fit(ks, ts)
        for K, t in zip(ks, ts):
            print(json.dumps({"impl": tag, "M": a.m, "N": a.n, "K": K, "us": round(t, 1),
                              "PFps": round(2 * a.m * a.n * K / t / 1e9, 3)}), flush=True)
        tiles = ((a.m + 255) // 256) * ((a.n + 255) // 256)
        waves = tiles / 256
        print(json.dumps({"impl": tag, "fit_fixed_us": round(f, 1), "fit_us_per_1k_K": round(b * 1024, 2),
                          "fixed_us_per_tile_wave": round(f / waves, 2),
                          "loop_PFps": round(2 * a.m * a.n / (b * 1e9), 3)}), flush=True)


if __name__ == "__main__":
    main()
