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
    ap.add_argument("--orders", default="seq", help="q-block orders to time (ops.prefill_qblocks order)")
    ap.add_argument("--hq", type=int, default=32, help="query heads (64: Llama-3-70B at TP=1)")
    ap.add_argument("--hkv", type=int, default=8)
    a = ap.parse_args()
    Hq, Hkv, D = a.hq, a.hkv, 128
    T = a.seqs * a.len
    qkv = torch.randn(T, (Hq + 2 * Hkv) * D, device="cuda", dtype=torch.bfloat16)
    cu = torch.arange(0, T + 1, a.len, dtype=torch.int32, device="cuda")
    qs, st = ops.prefill_qblocks(cu.tolist())
    qb = (torch.tensor(qs, dtype=torch.int32, device="cuda"), torch.tensor(st, dtype=torch.int32, device="cuda"))
    out = torch.empty(T, Hq * D, device="cuda", dtype=torch.bfloat16)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    flops = 4 * D * Hq * a.seqs * a.len * a.len / 2
    if os.environ.get("PLAIN", "1") == "1":  # the plain (cache-less) kernel
        for _ in range(3):
            ops.flash_prefill(qkv, cu, Hq, Hkv, D, D ** -0.5, qblocks=qb, out=out)
        torch.cuda.synchronize()
        e0.record()
        for _ in range(a.iters):
            ops.flash_prefill(qkv, cu, Hq, Hkv, D, D ** -0.5, qblocks=qb, out=out)
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) / a.iters * 1e3
        print(json.dumps({"seqs": a.seqs, "len": a.len, "kernel": "plain", "us": round(us, 1),
                          "PFps": round(flops / us / 1e9, 3)}))
    # paged (the engine's path): keys / values from a block-permuted cache, the v2 kernel
    bs = 16
    nb = a.seqs * ((a.len + bs - 1) // bs)
    kc = torch.zeros(nb + 4, Hkv, D // 8, bs, 8, device="cuda", dtype=torch.bfloat16)
    vc = torch.zeros(nb + 4, Hkv, D, bs, device="cuda", dtype=torch.bfloat16)
    per = (a.len + bs - 1) // bs
    bt = torch.randperm(nb, device="cuda").to(torch.int32).view(a.seqs, per)
    bt = torch.cat([bt, torch.zeros(a.seqs, 8, dtype=torch.int32, device="cuda")], 1).contiguous()
    pos = torch.arange(a.len, device="cuda").repeat(a.seqs).to(torch.int32)
    seq_of = torch.arange(a.seqs, device="cuda").repeat_interleave(a.len)
    slots = (bt[seq_of, (pos // bs).long()] * bs + pos % bs).to(torch.int32)
    ops.rope_and_cache(qkv, pos, torch.zeros(1, D, device="cuda"), kc, vc, slots, Hq, Hkv, D, apply_rope=False)
    cst = torch.zeros(a.seqs, dtype=torch.int32, device="cuda")
    res: dict = {}
    qbo = {}
    for order in a.orders.split(","):
        qs, st = ops.prefill_qblocks(cu.tolist(), order=order)
        qbo[order] = (torch.tensor(qs, dtype=torch.int32, device="cuda"),
                      torch.tensor(st, dtype=torch.int32, device="cuda"))
    for _ in range(3):
        for order in qbo:
            tag = f"paged_v2_{order}"
            qb = qbo[order]
            for _ in range(3):
                ops.flash_prefill(qkv, cu, Hq, Hkv, D, D ** -0.5, qblocks=qb, out=out, paged=(cst, kc, vc, bt))
            torch.cuda.synchronize()
            e0.record()
            for _ in range(a.iters):
                ops.flash_prefill(qkv, cu, Hq, Hkv, D, D ** -0.5, qblocks=qb, out=out, paged=(cst, kc, vc, bt))
            e1.record()
            torch.cuda.synchronize()
            res.setdefault(tag, []).append(e0.elapsed_time(e1) / a.iters * 1e3)
    for tag, ts in res.items():
        us = min(ts)
        print(json.dumps({"seqs": a.seqs, "len": a.len, "hq": Hq, "hkv": Hkv, "kernel": tag, "us": round(us, 1),
                          "PFps": round(flops / us / 1e9, 3)}))


if __name__ == "__main__":
    main()
