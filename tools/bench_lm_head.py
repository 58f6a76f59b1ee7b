"""Decode LM head of Llama-3-8B (N = 128256, K = 4096): hipBLASLt ``F.linear`` on the complete,
row-major final norm versus gemm_skinny_rm_kernel on the deferred-norm packed activation
(``skinny_linear`` with ``rownorm``).  hipGraph-captured calls, two weight copies rotated (2.1 GB,
so the weight streams from HBM), interleaved rounds.

    python tools/bench_lm_head.py [--ms 1,16,64] [--rounds 3]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from k8s_llm_monitor_amd import ops  # noqa: E402
from tools.bench_skinny import timeit  # noqa: E402


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=64)
    ap.add_argument("--ms", default="1,16,64")
    ap.add_argument("--rounds", type=int, default=3)
    a = ap.parse_args()
    dev = "cuda"
    V, d = 128256, 4096
    ws = [torch.randn(V, d, device=dev, dtype=torch.bfloat16) * 0.02 for _ in range(2)]
    nw = torch.rand(d, device=dev, dtype=torch.bfloat16) + 0.5
    gb = V * d * 2 / 1e9
    for M in map(int, a.ms.split(",")):
        res = torch.randn(M, d, device=dev, dtype=torch.bfloat16)
        x = ops.rms_norm(res, nw, 1e-5)
        xw, ss = ops.add_norm_partial(res.clone(), None, 0, nw)
        out = torch.empty(M, V, device=dev, dtype=torch.bfloat16)
        # parity first: the skinny path against the library on the same rows
        y_ref = F.linear(x, ws[0]).float()
        y_sk = ops.skinny_linear(xw, ws[0], rows=M, rownorm=(ss, 1e-5)).float()
        err = ((y_sk - y_ref).abs().max() / y_ref.abs().max()).item()
        agree = (y_sk.argmax(1) == y_ref.argmax(1)).float().mean().item()
        t: dict = {}
        for _ in range(a.rounds):
            t.setdefault("hipblaslt", []).append(timeit(lambda i: F.linear(x, ws[i % 2]), a.iters))
            t.setdefault("skinny_rm", []).append(timeit(
                lambda i: ops.skinny_linear(xw, ws[i % 2], out=out, rows=M, rownorm=(ss, 1e-5)), a.iters))
        for tag, ts in t.items():
            us = min(ts)
            print(json.dumps({"op": "lm_head", "M": M, "impl": tag, "us": round(us, 2),
                              "us_all": [round(v, 2) for v in ts], "TBps": round(gb / us * 1e3, 2),
                              "rel_err": round(err, 5), "argmax_agree": agree}), flush=True)


if __name__ == "__main__":
    main()
