"""The decode o projection's tail at M rows, three ways (one process, interleaved rounds, 32
hipGraph-captured calls rotating over > 512 MiB of weight copies so weights stream from HBM):
  slabs  - gemm_dec split-K slabs (8) + add_norm_partial (the r04 path),
  rc     - gemm_dec_rc_kernel: row-complete GEMM with the residual add and the next GEMM's
           deferred-norm operands in its epilogue,
and each followed by the gate_up + SwiGLU GEMM that consumes the normed rows (per-512-column
partials vs per-16-column partials), so the consumer's side of the change is timed too.

    python tools/bench_dec_rc.py [--ms 1,32,64] [--rounds 3]
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

D, FF = 4096, 14336


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=320)
    ap.add_argument("--ms", default="1,32,64")
    ap.add_argument("--rounds", type=int, default=3)
    a = ap.parse_args()
    dev = "cuda"
    torch.manual_seed(0)
    ncopy = (512 << 20) // ((D * D + 2 * FF * D) * 2) + 2
    wo = [ops.pack_skinny(torch.randn(D, D, device=dev, dtype=torch.bfloat16) * 0.02) for _ in range(ncopy)]
    wgu = [ops.pack_skinny(ops.interleave_gate_up8(torch.randn(2 * FF, D, device=dev, dtype=torch.bfloat16) * 0.02))
           for _ in range(ncopy)]
    nw = torch.ones(D, device=dev, dtype=torch.bfloat16)
    for M in map(int, a.ms.split(",")):
        x = ops.pack_activation(torch.randn(M, D, device=dev, dtype=torch.bfloat16))
        resid = torch.randn(M, D, device=dev, dtype=torch.bfloat16)
        ws = torch.empty(8 * M * D, device=dev)
        act = ops.packed_empty(M, FF, torch.bfloat16, dev)
        xw = ops.packed_empty(M, D, torch.bfloat16, dev)
        ss8 = torch.empty(M, D // 512, device=dev)
        xw_rc = ops.packed_empty(M, D, torch.bfloat16, dev)
        ss256 = torch.empty(M, D // 16, device=dev)

        def slabs(i, gu):
            s = ops.dec_gemm(x, wo[i % ncopy], 0, M, workspace=ws)
            ops.add_norm_partial(resid, ws, s, nw, out=xw, ss_part=ss8)
            if gu:
                ops.dec_gemm(xw, wgu[i % ncopy], 2, M, out=act, rownorm=(ss8, 1e-5))

        def rc(i, gu):
            ops.native().gemm_dec_rc(x, wo[i % ncopy], resid, nw, xw_rc, ss256, M)
            if gu:
                ops.dec_gemm(xw_rc, wgu[i % ncopy], 2, M, out=act, rownorm=(ss256, 1e-5))

        cases = {"slabs": lambda i: slabs(i, False), "rc": lambda i: rc(i, False),
                 "slabs+gu": lambda i: slabs(i, True), "rc+gu": lambda i: rc(i, True)}
        res: dict = {}
        for _ in range(a.rounds):
            for tag, fn in cases.items():
                res.setdefault(tag, []).append(timeit(fn, a.iters))
        for tag, ts in res.items():
            print(json.dumps({"M": M, "impl": tag, "us": round(min(ts), 2), "us_all": [round(v, 2) for v in ts]}),
                  flush=True)


if __name__ == "__main__":
    main()
