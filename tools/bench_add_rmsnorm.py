"""Fused residual add + RMSNorm at the prefill chunk shape (16384 x 4096): us and TB/s.

    python tools/bench_add_rmsnorm.py [--rows 16384] [--d 4096]
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
    ap.add_argument("--d", type=int, default=4096)
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    x = torch.randn(a.rows, a.d, device="cuda", dtype=torch.bfloat16)
    r = torch.randn(a.rows, a.d, device="cuda", dtype=torch.bfloat16)
    w = torch.randn(a.d, device="cuda", dtype=torch.bfloat16)
    for _ in range(3):
        ops.fused_add_rms_norm(x, r, w, 1e-5)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(a.iters):
        ops.fused_add_rms_norm(x, r, w, 1e-5)
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) / a.iters * 1e3
    print(json.dumps({"rows": a.rows, "d": a.d, "us": round(us, 1), "TBps": round(a.rows * a.d * 8 / us / 1e6, 2)}))


if __name__ == "__main__":
    main()
