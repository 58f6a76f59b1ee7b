"""Does a decode projection run faster when its weights were just streamed through the Infinity
Cache (MALL) by another kernel?  qkv / o shared-A decode GEMMs at M = 64: cold (the previous call
used another weight copy, > 512 MiB rotated) vs warm (a read-only pass over the same packed weight
right before), device time of the GEMM alone by events.  Feasibility probe for a side-stream
weight prefetch in the decode graph.

    python tools/probe_mall_warm.py
"""
from __future__ import annotations

import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from k8s_llm_monitor_amd import ops  # noqa: E402


def main() -> None:
    dev = "cuda"
    torch.manual_seed(0)
    M = 64
    for name, (N, K) in (("qkv", (6144, 4096)), ("o", (4096, 4096)), ("down", (4096, 14336))):
        ncopy = max(2, (768 << 20) // (N * K * 2) + 1)
        wps = [ops.pack_skinny(torch.randn(N, K, device=dev, dtype=torch.bfloat16) * 0.02) for _ in range(ncopy)]
        x = ops.pack_activation(torch.randn(M, K, device=dev, dtype=torch.bfloat16))
        ws = torch.empty(16 * M * N, device=dev, dtype=torch.float32)
        sink = torch.empty(1, device=dev, dtype=torch.float32)
        res = {"cold": [], "warm": []}
        for it in range(40):
            i = it % ncopy
            warm = it % 2 == 1
            if warm:  # read the same weights through the caches just before (a reduction kernel)
                sink.copy_(wps[i].view(torch.int32).sum(dtype=torch.int64).float().view(1))
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            ops.dec_gemm(x, wps[i], 0, M, workspace=ws)
            e1.record()
            torch.cuda.synchronize()
            if it >= 4:
                res["warm" if warm else "cold"].append(e0.elapsed_time(e1) * 1e3)
        print(json.dumps({"op": name, "M": M, "cold_us": round(sorted(res["cold"])[len(res["cold"]) // 2], 2),
                          "warm_us": round(sorted(res["warm"])[len(res["warm"]) // 2], 2)}), flush=True)


if __name__ == "__main__":
    main()
