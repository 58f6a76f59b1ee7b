"""Flash prefill attention on the bench's prefill shape (Llama-3-8B heads: Hq 32, Hkv 8, D 128):
``--seqs`` sequences of ``--len`` tokens in one varlen batch; prints us per call and PF/s
(causal FLOPs = 4 * D * Hq * sum(L^2 / 2)).

    python tools/bench_prefill_attn.py [--seqs 10] [--len 1609]
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
    ap.add_argument("--seqs", type=int, default=10)
    ap.add_argument("--len", type=int, default=1609)
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    Hq, Hkv, D = 32, 8, 128
    T = a.seqs * a.len
    qkv = torch.randn(T, (Hq + 2 * Hkv) * D, device="cuda", dtype=torch.bfloat16)
    cu = torch.arange(0, T + 1, a.len, dtype=torch.int32, device="cuda")
    qs, st = ops.prefill_qblocks(cu.tolist())
    qb = (torch.tensor(qs, dtype=torch.int32, device="cuda"), torch.tensor(st, dtype=torch.int32, device="cuda"))
    out = torch.empty(T, Hq * D, device="cuda", dtype=torch.bfloat16)
    for _ in range(3):
        ops.flash_prefill(qkv, cu, Hq, Hkv, D, D ** -0.5, qblocks=qb, out=out)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(a.iters):
        ops.flash_prefill(qkv, cu, Hq, Hkv, D, D ** -0.5, qblocks=qb, out=out)
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) / a.iters * 1e3
    flops = 4 * D * Hq * a.seqs * a.len * a.len / 2
    print(json.dumps({"seqs": a.seqs, "len": a.len, "us": round(us, 1), "PFps": round(flops / us / 1e9, 3)}))


if __name__ == "__main__":
    main()
