"""Decode LM head (Llama-3-8B: V 128256 x d 4096, 1.05 GB bf16) at decode batch sizes: hipBLASLt
(F.linear on row-major activations) versus the row-major skinny GEMM (fragment-packed A, the
weight streamed by LDS-DMA), 32 graph-replayed calls, interleaved rounds.

    python tools/bench_lm_head.py [--ms 1,16,64]
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
    ap.add_argument("--ms", default="1,16,64")
    a = ap.parse_args()
    V, d = 128256, 4096
    w = torch.randn(V, d, device="cuda", dtype=torch.bfloat16) * 0.02
    gb = V * d * 2 / 1e9
    for M in map(int, a.ms.split(",")):
        x = torch.randn(M, d, device="cuda", dtype=torch.bfloat16)
        xp = ops.pack_activation(x)
        y = torch.empty(M, V, device="cuda", dtype=torch.bfloat16)
        ref = torch.nn.functional.linear(x, w)
        got = ops.skinny_linear(xp, w, rows=M)
        err = float((ref.float() - got.float()).abs().max())
        res: dict = {}
        for _ in range(3):
            res.setdefault("hipblaslt", []).append(timeit(lambda i: torch.nn.functional.linear(x, w, out=y)
                                                          if False else torch.mm(x, w.t(), out=y), 64))
            res.setdefault("skinny_rm", []).append(timeit(lambda i: ops.skinny_linear(xp, w, out=y, rows=M), 64))
        for k, ts in res.items():
            t = min(ts)
            print(json.dumps({"M": M, "impl": k, "us": round(t, 2), "TBps": round(gb / t * 1e3, 2),
                              "max_abs_diff": round(err, 4)}), flush=True)


if __name__ == "__main__":
    main()
