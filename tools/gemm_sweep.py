"""Decode/prefill GEMM shapes of Llama-3-8B: default hipBLASLt vs rocBLAS vs TunableOp-tuned.

    python tools/gemm_sweep.py [--tune]   (writes profiles/tunableop_*.csv when tuning)
"""
import os
import sys
import time

import torch
import torch.nn.functional as F

SHAPES = {"qkv": (6144, 4096), "o": (4096, 4096), "gate_up": (28672, 4096), "down": (4096, 14336),
          "lm_head": (128256, 4096)}
MS = [int(m) for m in os.environ.get("MS", "1,8,32,64,128,8192").split(",")]


def bench(fn, n=30):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(True), torch.cuda.Event(True)
    e0.record()
    for _ in range(n):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / n * 1e3


def main():
    torch.manual_seed(0)
    libs = sys.argv[1:] or ["default", "cublas"]
    res = {}
    for lib in libs:
        if lib in ("cublas", "cublaslt"):
            torch.backends.cuda.preferred_blas_library(lib)
        for name, (N, K) in SHAPES.items():
            w = torch.randn(N, K, device="cuda", dtype=torch.bfloat16) * 0.02
            for M in MS:
                if name == "lm_head" and M > 128:
                    continue
                x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
                t = bench(lambda: F.linear(x, w))
                res[(lib, name, M)] = t
            del w
    for name, (N, K) in SHAPES.items():
        for M in MS:
            row = [res.get((lib, name, M)) for lib in libs]
            if row[0] is None:
                continue
            wb = N * K * 2
            cells = "  ".join(f"{lib}={t:8.1f}us ({wb / t / 1e6:5.2f}TB/s, {2 * M * N * K / t / 1e6:7.1f}TF)" for lib, t in zip(libs, row))
            print(f"{name:8s} M={M:6d} N={N:6d} K={K:6d}  {cells}", flush=True)


if __name__ == "__main__":
    main()
