"""Row-major skinny GEMM decode projections (Llama-3-8B, M = 64): split-K x waves-per-workgroup
sweep (32 graph-replayed calls over > 512 MiB of weight copies, min of 3 interleaved rounds).

    python tools/bench_skinny_rm_splits.py [--m 64]
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


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--m", type=int, default=64)
    a = ap.parse_args()
    d, F = 4096, 14336
    M = a.m
    shapes = {"qkv": (6144, d, (1, 2, 3, 4, 6, 8)), "o": (d, d, (2, 4, 8)), "down": (d, F, (2, 4, 7, 8))}
    for name, (N, K, splits) in shapes.items():
        ncopy = max(2, (512 << 20) // (N * K * 2) + 1)
        wrm = [torch.randn(N, K, device="cuda", dtype=torch.bfloat16) * 0.02 for _ in range(ncopy)]
        xp = ops.pack_activation(torch.randn(M, K, device="cuda", dtype=torch.bfloat16))
        ws = ops.skinny_workspace(M, N, 16, "cuda")
        res: dict = {}
        for _ in range(3):
            for s in splits:
                for wv in ("2", "4"):
                    ops.SKINNY_WAVES_FORCE = int(wv)
                    res.setdefault((s, wv), []).append(
                        timeit(lambda i, s=s: ops.skinny_slabs(xp, wrm[i % ncopy], ws, s, rows=M), 320))
        ops.SKINNY_WAVES_FORCE = 0
        for (s, wv), ts in sorted(res.items()):
            t = min(ts)
            print(json.dumps({"op": name, "M": M, "splits": s, "waves": int(wv), "us": round(t, 2),
                              "TBps": round(N * K * 2 / t / 1e6, 2)}), flush=True)
        del wrm
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
