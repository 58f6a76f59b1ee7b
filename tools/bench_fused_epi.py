"""Fused skinny epilogues vs the slab + reduce-kernel pairs they replace, Llama-3-8B decode shapes
(M = 64 rows), timed as hipGraph-captured sequences rotating over > 512 MiB of weight copies
(weights stream from HBM, as in a 32-layer decode step).  Times include the reduce kernel for
the unfused pairs, i.e. the per-layer cost the decode step pays.

  o / down : skinny_slabs (auto split-K) + add_norm_partial   vs  skinny_resnorm (split-K, waves 4/8)
  qkv      : skinny_slabs (auto split-K, rownorm) + rope_and_cache  vs  skinny_qkv_rope (split-K, waves 4/8)

    python tools/bench_fused_epi.py [--ms 64]
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
from tools.bench_skinny import timeit  # noqa: E402


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=320)
    ap.add_argument("--ms", default="64")
    ap.add_argument("--ops", default="qkv,o,down")
    ap.add_argument("--layout", default="rowmajor", choices=["rowmajor", "packed"],
                    help="weight layout: the engine's row-major tensors (default) or fragment-packed copies")
    a = ap.parse_args()
    dev = "cuda"
    d, F, hq, hkv, D, bs = 4096, 14336, 32, 8, 128, 16
    shapes = {"qkv": ((hq + 2 * hkv) * D, d), "o": (d, d), "down": (d, F)}
    nw = (torch.rand(d, device=dev) + 0.5).to(torch.bfloat16)
    cs = ref.rope_cos_sin(8192, D, 500000.0, None, device=dev)
    for name in a.ops.split(","):
        N, K = shapes[name]
        ncopy = max(2, (512 << 20) // (N * K * 2) + 1)
        keep = ops.pack_skinny if a.layout == "packed" else (lambda w: w)
        wps = [keep(torch.randn(N, K, device=dev, dtype=torch.bfloat16) * 0.02) for _ in range(ncopy)]
        gb = N * K * 2 / 1e9
        for M in map(int, a.ms.split(",")):
            xp = ops.pack_activation(torch.randn(M, K, device=dev, dtype=torch.bfloat16))
            ws = ops.skinny_workspace(M, max(N, d), 16, dev)
            res = torch.randn(M, d, device=dev, dtype=torch.bfloat16)
            cases = []
            if name == "qkv":
                ssk = torch.rand(M, K // 512, device=dev) * K
                qkv = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
                nb = 4 * M
                kc = torch.zeros(nb, hkv, D // 8, bs, 8, device=dev, dtype=torch.bfloat16)
                vc = torch.zeros(nb, hkv, D, bs, device=dev, dtype=torch.bfloat16)
                pos = torch.randint(0, 2000, (M,), dtype=torch.int32, device=dev)
                slots = torch.randperm(nb * bs, device=dev)[:M].to(torch.int32)

                def old(i):
                    ns = ops.skinny_slabs(xp, wps[i % ncopy], ws, 0, rows=M, rownorm=(ssk, 1e-5))
                    ops.rope_and_cache(qkv, pos, cs, kc, vc, slots, hq, hkv, D, partial=ws, nslabs=ns)

                cases.append(("slabs+rope", "0", old))
                for sp in (0, 2, 4):
                    for waves in ("4", "8"):
                        cases.append((f"fused_s{sp}_w{waves}", waves,
                                      lambda i, sp=sp: ops.skinny_qkv_rope(xp, wps[i % ncopy], qkv, pos, cs, kc, vc,
                                                                           slots, hq, hkv, rows=M, rownorm=(ssk, 1e-5),
                                                                           workspace=ws, splits=sp)))
            else:
                out = ops.packed_empty(M, d, torch.bfloat16, dev)
                ss4 = torch.empty(M, d // 64, device=dev)
                ssp = torch.empty(M, d // 512, device=dev)

                def old(i):
                    ns = ops.skinny_slabs(xp, wps[i % ncopy], ws, 0, rows=M)
                    ops.add_norm_partial(res, ws, ns, nw, out=out, ss_part=ssp)

                cases.append(("slabs+add_norm", "0", old))
                for sp in (0, 2, 4, 8):
                    for waves in ("4", "8"):
                        cases.append((f"resnorm_s{sp}_w{waves}", waves,
                                      lambda i, sp=sp: ops.skinny_resnorm(xp, wps[i % ncopy], res, nw, rows=M, out=out,
                                                                          ss=ss4, workspace=ws, splits=sp)))
            for tag, waves, fn in cases:
                os.environ["K8SLLM_SKINNY_WAVES"] = waves
                t = timeit(fn, a.iters)
                print(json.dumps({"op": name, "M": M, "impl": tag, "us": round(t, 2),
                                  "TBps_weights": round(gb / t * 1e3, 2)}), flush=True)
            os.environ["K8SLLM_SKINNY_WAVES"] = "0"
        del wps
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
