"""Decode residual-add + deferred-norm pass (add_norm_partial) at Llama-3-8B width: graph-replayed
calls over the split-K slab counts the decode GEMMs produce.  Run once per K8SLLM_ANP_STATIC
setting (read once per process).

    python tools/bench_add_norm.py
"""
from __future__ import annotations

import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from k8s_llm_monitor_amd import ops  # noqa: E402
from tools.bench_skinny import timeit  # noqa: E402


def main() -> None:
    dev, d = "cuda", 4096
    nw = (torch.rand(d, device=dev) + 0.5).to(torch.bfloat16)
    for M in (1, 64):
        for S in (2, 4):
            res = torch.randn(M, d, device=dev, dtype=torch.bfloat16)
            ws = torch.randn(S * M * d, device=dev, dtype=torch.float32)
            ref = (res.float() + ws.view(S, M, d).sum(0)).to(torch.bfloat16)
            r2 = res.clone()
            xw, ss = ops.add_norm_partial(r2, ws, S, nw)
            ok = bool((r2.float() - ref.float()).abs().max() < 1e-2) and bool(
                (ss.sum(1) - (ref.float() ** 2).sum(1)).abs().max() < 1e-2 * (ref.float() ** 2).sum(1).max())
            out = ops.packed_empty(M, d, torch.bfloat16, dev)
            sp = torch.empty_like(ss)
            us = min(timeit(lambda i: ops.add_norm_partial(res, ws, S, nw, out=out, ss_part=sp), 320) for _ in range(3))
            print(json.dumps({"op": "add_norm_partial", "M": M, "S": S, "static": os.environ.get("K8SLLM_ANP_STATIC", "1"),
                              "us": round(us, 2), "parity_ok": ok}), flush=True)


if __name__ == "__main__":
    main()
