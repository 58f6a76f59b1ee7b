"""Decode projections of a Llama-3-8B layer: gemm_skinny over the fragment-packed weight copy
versus gemm_skinny_rm_kernel over the row-major weight itself (LDS-DMA whole-line staging), in
one process, interleaved rounds (cdna_hip_programming.md §5.4 rule 24).  Each case is 32
hipGraph-captured calls rotating over > 512 MiB of weight copies (weights stream from HBM).

    python tools/bench_skinny_rm.py [--ms 1,16,64] [--rounds 3]
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
    ap.add_argument("--iters", type=int, default=320)
    ap.add_argument("--ms", default="1,16,64")
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--ops", default="qkv,o,gate_up,down")
    ap.add_argument("--ncopy", type=int, default=0, help="weight copies rotated (0: enough for > 512 MiB)")
    ap.add_argument("--impls", default="packed,rowmajor,rowmajor_w2,rowmajor_w4")
    a = ap.parse_args()
    dev = "cuda"
    d, F = 4096, 14336
    shapes = {"qkv": (6144, d), "o": (d, d), "gate_up": (2 * F, d), "down": (d, F),
              "gate_up_32k": (32768, d), "gate_up_24k": (24576, d)}  # balance probes: 512 / 384 workgroups
    for name in a.ops.split(","):
        N, K = shapes[name]
        ncopy = a.ncopy or max(2, (512 << 20) // (N * K * 2) + 1)
        wrm = [(torch.randn(N, K, device=dev, dtype=torch.bfloat16) * 0.02) for _ in range(ncopy)]
        wpk = [ops.pack_skinny(w) for w in wrm]
        gb = N * K * 2 / 1e9
        for M in map(int, a.ms.split(",")):
            xp = ops.pack_activation(torch.randn(M, K, device=dev, dtype=torch.bfloat16))
            act = ops.packed_empty(M, N // 2, torch.bfloat16, dev)
            wsp = ops.skinny_workspace(M, N, 16, dev)
            res: dict = {}
            tag_sfx = f"_ncopy{ncopy}"
            for _ in range(a.rounds):
                for tag, ws_, wv in (("packed", wpk, "0"), ("rowmajor", wrm, "0"), ("rowmajor_w2", wrm, "2"),
                                     ("rowmajor_w4", wrm, "4")):
                    if tag not in a.impls.split(","):
                        continue
                    ops.SKINNY_WAVES_FORCE = int(wv)
                    if name.startswith("gate_up"):
                        fn = (lambda i, ws_=ws_: ops.skinny_swiglu(xp, ws_[i % ncopy], out=act, rows=M, packed_out=True))
                    else:
                        fn = (lambda i, ws_=ws_: ops.skinny_slabs(xp, ws_[i % ncopy], wsp, 0, rows=M))
                    res.setdefault(tag, []).append(timeit(fn, a.iters))
            for tag, ts in res.items():
                t = min(ts)
                print(json.dumps({"op": name, "M": M, "impl": tag + tag_sfx, "us": round(t, 2), "us_all": [round(x, 2) for x in ts],
                                  "TBps": round(gb / t * 1e3, 2)}), flush=True)
        del wrm, wpk
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
