"""gemm_skinny alone (no reduce), the engine's decode calls for Llama-3-8B, swept over waves per
workgroup (4 / 8) and split-K factor.  Timed as 32 hipGraph-captured calls rotating over > 512 MiB
of weight copies (weights stream from HBM, as in a 32-layer decode step).

    python tools/bench_skinny_waves.py [--ms 64] [--splits 0,2,3,4,6,8]
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
    ap.add_argument("--ms", default="64")
    ap.add_argument("--splits", default="0,2,3,4,6,8")
    ap.add_argument("--ops", default="qkv,o,gate_up,down")
    a = ap.parse_args()
    dev = "cuda"
    d, F = 4096, 14336
    shapes = {"qkv": (6144, d), "o": (d, d), "gate_up": (2 * F, d), "down": (d, F)}
    for name in a.ops.split(","):
        N, K = shapes[name]
        ncopy = max(2, (512 << 20) // (N * K * 2) + 1)
        wps = [ops.pack_skinny(torch.randn(N, K, device=dev, dtype=torch.bfloat16) * 0.02) for _ in range(ncopy)]
        gb = N * K * 2 / 1e9
        for M in map(int, a.ms.split(",")):
            xp = ops.pack_activation(torch.randn(M, K, device=dev, dtype=torch.bfloat16))
            act = ops.packed_empty(M, F, torch.bfloat16, dev)
            wsp = ops.skinny_workspace(M, N, 16, dev)
            for waves in ("4", "8"):
                ops.SKINNY_WAVES_FORCE = int(waves)
                if name == "gate_up":
                    cases = [("swiglu", lambda i: ops.skinny_swiglu(xp, wps[i % ncopy], out=act, rows=M,
                                                                   packed_out=True))]
                else:
                    cases = [(f"s{s}", lambda i, s=s: ops.skinny_slabs(xp, wps[i % ncopy], wsp, s, rows=M))
                             for s in map(int, a.splits.split(","))]
                for tag, fn in cases:
                    t = timeit(fn, a.iters)
                    print(json.dumps({"op": name, "M": M, "waves": int(waves), "impl": tag, "us": round(t, 2),
                                      "TBps": round(gb / t * 1e3, 2)}), flush=True)
        del wps
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
