"""Decode projections of a Llama-3-8B layer (+ the LM head) at decode batch M: the shipped
row-major skinny kernel (gemm_skinny_rm_kernel; hipBLASLt F.linear for the LM head) against the
shared-A decode GEMM (gemm_decode.hip) over its packed weight copies, for a list of launch
configurations (splits, n-tiles per wave, waves, ring depth).  One process, interleaved rounds;
each case is 32 hipGraph-captured calls rotating over > 512 MiB of weight copies, so weights
stream from HBM as in a decode step.  Every dec configuration is checked against an fp32
reference of the same product first (max |err| / max |ref|).

    python tools/bench_decode_gemm.py [--ms 1,32,64] [--ops qkv,o,gate_up,down,lm_head] [--rounds 3]
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

D, FF, V = 4096, 14336, 128256
SHAPES = {"qkv": (6144, D, 0), "o": (D, D, 0), "gate_up": (2 * FF, D, 2), "down": (D, FF, 0), "lm_head": (V, D, 1)}
CFGS = {  # configurations gemm_decode.hip instantiates (other sweeps: add the instantiation first)
    "qkv": [(4, 1, 6, 8), (8, 1, 8, 8), (4, 1, 4, 16), (4, 1, 4, 8)],
    "o": [(4, 1, 4, 16), (4, 1, 4, 8), (8, 1, 8, 8), (16, 1, 8, 8)],
    "gate_up": [(1, 1, 7, 16), (1, 1, 7, 8), (1, 1, 8, 16)],
    "down": [(4, 1, 4, 16), (4, 1, 4, 8), (8, 1, 8, 8), (4, 1, 8, 8)],
    "lm_head": [(1, 4, 8, 4), (1, 3, 8, 8), (1, 2, 8, 8)],
}


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=320)
    ap.add_argument("--ms", default="1,32,64")
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--ops", default="qkv,o,gate_up,down,lm_head")
    ap.add_argument("--cfgs", default=None, help="op:S,NTW,W,D|S,NTW,W,D;... overrides the sweep list")
    a = ap.parse_args()
    dev = "cuda"
    torch.manual_seed(0)
    cfgs = dict(CFGS)
    if a.cfgs:
        for item in a.cfgs.split(";"):
            op, c = item.split(":")
            cfgs[op] = [tuple(int(v) for v in cc.split(",")) for cc in c.split("|")]
    for name in a.ops.split(","):
        N, K, epi = SHAPES[name]
        ncopy = max(2, (512 << 20) // (N * K * 2) + 1)
        wrm = [(torch.randn(N, K, device=dev, dtype=torch.bfloat16) * 0.02) for _ in range(ncopy)]
        if epi == 2:  # the engine's resident w13 is [64 gate | 64 up]-interleaved; the dec copy by 8
            canon = [ops.deinterleave_gate_up(w) for w in wrm]
            wdec = [ops.pack_skinny(ops.interleave_gate_up8(w)) for w in canon]
        else:
            wdec = [ops.pack_skinny(w) for w in wrm]
        gb = N * K * 2 / 1e9
        for M in map(int, a.ms.split(",")):
            x = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
            xp = ops.pack_activation(x)
            ref = x.float() @ wrm[0].float().t()
            if epi == 2:
                g, u = ops._cpu_deinterleave(ref.to(torch.bfloat16).float())
                ref = F.silu(g) * u
            scale = ref.abs().max().item()
            wsp = torch.empty(16 * M * N, device=dev, dtype=torch.float32)
            act = ops.packed_empty(M, N // 2, torch.bfloat16, dev)
            yb = torch.empty(M, N, device=dev, dtype=torch.bfloat16)

            def dec_out(cfg):
                if epi == 0:
                    s = ops.dec_gemm(xp, wdec[0], 0, M, workspace=wsp, cfg=cfg)
                    return wsp[: s * M * N].view(s, M, N).sum(0)
                if epi == 1:
                    ops.dec_gemm(xp, wdec[0], 1, M, out=yb, cfg=cfg)
                    return yb.float()
                ops.dec_gemm(xp, wdec[0], 2, M, out=act, cfg=cfg)
                return ops.unpack_skinny(act)[:M].float()

            cases = {}
            if epi == 0:
                cases["rm"] = lambda i: ops.skinny_slabs(xp, wrm[i % ncopy], wsp, 0, rows=M)
            elif epi == 2:
                cases["rm"] = lambda i: ops.skinny_swiglu(xp, wrm[i % ncopy], out=act, rows=M, packed_out=True)
            else:
                cases["hipblaslt"] = lambda i: torch.matmul(x, wrm[i % ncopy].t(), out=yb)
            for cfg in cfgs[name]:
                try:
                    err = (dec_out(cfg) - ref).abs().max().item() / max(scale, 1e-6)
                except (RuntimeError, ValueError) as e:
                    print(json.dumps({"op": name, "M": M, "cfg": cfg, "error": str(e)[:200]}), flush=True)
                    continue
                tag = "dec" + "_".join(map(str, cfg))
                cases[tag] = (lambda i, cfg=cfg: ops.dec_gemm(xp, wdec[i % ncopy], epi, M, workspace=wsp,
                                                              out=act if epi == 2 else yb, cfg=cfg))
                print(json.dumps({"op": name, "M": M, "cfg": cfg, "rel_err": round(err, 5)}), flush=True)
            res: dict = {}
            for _ in range(a.rounds):
                for tag, fn in cases.items():
                    res.setdefault(tag, []).append(timeit(fn, a.iters))
            for tag, ts in res.items():
                t = min(ts)
                print(json.dumps({"op": name, "M": M, "impl": tag, "us": round(t, 2),
                                  "us_all": [round(v, 2) for v in ts], "TBps": round(gb / t * 1e3, 2)}), flush=True)
        del wrm, wdec
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
