"""Decode sampler timing: ops.sample over [B, V] bf16 logits (LM-head-like: x / T has std ~13 at
T = 0.1 for a random-init Llama-3-8B head) - greedy, T = 0.1, T = 1.0; hipGraph replay of
back-to-back calls.

    python tools/bench_sampler.py [--b 64] [--v 128256]
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
    ap.add_argument("--b", type=int, default=64)
    ap.add_argument("--v", type=int, default=128256)
    a = ap.parse_args()
    dev = "cuda"
    torch.manual_seed(0)
    logits = (torch.randn(a.b, a.v, device=dev) * 1.28).to(torch.bfloat16)
    out = torch.empty(a.b, dtype=torch.int32, device=dev)
    rng = torch.tensor([1, 0], device=dev, dtype=torch.int64)
    for name, t in (("greedy", 0.0), ("T0.1", 0.1), ("T1.0", 1.0)):
        temps = torch.full((a.b,), t, device=dev)
        us = timeit(lambda i: ops.sample(logits, temps, None, None, rng, out=out, advance=True), 64, per_graph=8)
        print(json.dumps({"op": "sample", "B": a.b, "V": a.v, "mode": name, "us": round(us, 2)}), flush=True)


if __name__ == "__main__":
    main()
