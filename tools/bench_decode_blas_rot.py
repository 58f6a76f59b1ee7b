"""hipBLASLt (torch.matmul) at decode shapes with weights ROTATING over > 512 MiB of copies, the
same methodology as tools/bench_skinny_waves.py (a single weight buffer of <= 256 MB is partly
served by the Infinity Cache and overstates HBM bandwidth) - for an apples-to-apples comparison of
the library GEMM with the skinny MFMA kernels; gate_up also timed with the separate silu_mul pass.

    python tools/bench_decode_blas_rot.py [--ms 1,64]
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
    a = ap.parse_args()
    dev = "cuda"
    d, F = 4096, 14336
    shapes = {"qkv": (6144, d), "o": (d, d), "gate_up": (2 * F, d), "down": (d, F), "lm_head": (128256, d)}
    for name, (N, K) in shapes.items():
        ncopy = max(2, (512 << 20) // (N * K * 2) + 1)
        ws = [torch.randn(N, K, device=dev, dtype=torch.bfloat16) * 0.02 for _ in range(ncopy)]
        gb = N * K * 2 / 1e9
        for M in map(int, a.ms.split(",")):
            x = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
            y = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
            t = timeit(lambda i: torch.matmul(x, ws[i % ncopy].t(), out=y), a.iters)
            print(json.dumps({"op": name, "M": M, "impl": "hipblaslt_rot", "us": round(t, 2),
                              "TBps": round(gb / t * 1e3, 2)}), flush=True)
            if name == "gate_up":
                act = torch.empty(M, F, device=dev, dtype=torch.bfloat16)

                def fn(i):
                    torch.matmul(x, ws[i % ncopy].t(), out=y)
                    ops.silu_mul(y, out=act)
                t = timeit(fn, a.iters)
                print(json.dumps({"op": name, "M": M, "impl": "hipblaslt_rot+silu_mul", "us": round(t, 2),
                                  "TBps": round(gb / t * 1e3, 2)}), flush=True)
        del ws
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
