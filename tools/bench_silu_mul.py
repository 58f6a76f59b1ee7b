"""silu_mul at the prefill chunk shape (16384 tokens x 14336 SwiGLU columns): us and TB/s.

    python tools/bench_silu_mul.py [--rows 16384] [--ff 14336]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from k8s_llm_monitor_amd import ops  # noqa: E402


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=16384)
    ap.add_argument("--ff", type=int, default=14336)
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    x = torch.randn(a.rows, 2 * a.ff, device="cuda", dtype=torch.bfloat16)
    out = torch.empty(a.rows, a.ff, device="cuda", dtype=torch.bfloat16)
    for _ in range(3):
        ops.silu_mul(x, out=out)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(a.iters):
        ops.silu_mul(x, out=out)
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) / a.iters * 1e3
    print(json.dumps({"rows": a.rows, "ff": a.ff, "us": round(us, 1), "TBps": round(a.rows * a.ff * 6 / us / 1e6, 2)}))


if __name__ == "__main__":
    main()
