"""Prefill rope_and_cache at the bench's chunk shape (Llama-3-8B heads, 12 x 1365 tokens): time
with the paged K/V cache write, without it (rope only), and the cache write alone.

    python tools/bench_rope_cache.py [--seqs 12] [--len 1365]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from k8s_llm_monitor_amd import ops  # noqa: E402
from k8s_llm_monitor_amd.ops import reference as ref  # noqa: E402


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--seqs", type=int, default=12)
    ap.add_argument("--len", type=int, default=1365)
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    Hq, Hkv, D, BS = 32, 8, 128, 16
    T = a.seqs * a.len
    dev = "cuda"
    qkv = torch.randn(T, (Hq + 2 * Hkv) * D, device=dev, dtype=torch.bfloat16)
    per = (a.len + BS - 1) // BS
    nb = a.seqs * per + 4
    kc = torch.zeros(nb, Hkv, D // 8, BS, 8, device=dev, dtype=torch.bfloat16)
    vc = torch.zeros(nb, Hkv, D, BS, device=dev, dtype=torch.bfloat16)
    pos = torch.arange(a.len, device=dev, dtype=torch.int32).repeat(a.seqs)
    blocks = torch.randperm(nb, device=dev)[: a.seqs * per].view(a.seqs, per).to(torch.int32)
    slots = (blocks[:, :, None] * BS + torch.arange(BS, device=dev, dtype=torch.int32)).view(a.seqs, -1)[:, : a.len]
    slots = slots.reshape(-1).contiguous()
    cs = ref.rope_cos_sin(8192, D, 500000.0, None, device=dev)
    nbytes = {"cache": T * ((Hq + 2 * Hkv) * D * 2 + (Hq + Hkv) * D * 2 + 2 * Hkv * D * 2),
              "rope_only": T * (Hq + Hkv) * D * 2 * 2, "cache_only": T * 2 * Hkv * D * 2 * 2}
    cases = {"cache": (slots, True), "rope_only": (None, True), "cache_only": (slots, False)}
    out = {"T": T}
    for name, (sl, rope) in cases.items():
        for _ in range(3):
            ops.rope_and_cache(qkv, pos, cs, kc, vc, sl, Hq, Hkv, D, apply_rope=rope)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(a.iters):
            ops.rope_and_cache(qkv, pos, cs, kc, vc, sl, Hq, Hkv, D, apply_rope=rope)
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) / a.iters * 1e3
        out[name] = {"us": round(us, 1), "TBps": round(nbytes[name] / us / 1e6, 2)}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
