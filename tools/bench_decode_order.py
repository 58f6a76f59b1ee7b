"""Does the order of the batch rows matter for paged decode attention at ragged contexts?

Batch 64 x 8 kv heads = 512 workgroups, two per CU: WG z of an XCD shares a CU with (probably) WG
z + 32.  Contexts drawn like the headline wave (prompts 1.2k-2.2k tokens + up to 256 generated).
Orders: random, paired (row z and row z + 32 = the k-th longest and the k-th shortest), sorted
longest-first, sorted shortest-first.  Prints one JSON line per order (min over rounds)."""
import json
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from k8s_llm_monitor_amd import ops

torch.manual_seed(0)
DEV = "cuda"
hq, hkv, d, bs = 32, 8, 128, 16
B = 64
g = torch.Generator().manual_seed(1)
lens_list = [int(x) for x in torch.randint(1200, 2200, (B,), generator=g) + 128]
maxlen = 8192
mb = maxlen // bs
pers = [ln // bs + 1 for ln in lens_list]
nb = sum(pers) + 8
kc = torch.randn(nb, hkv, d // 8, bs, 8, device=DEV, dtype=torch.bfloat16)
vc = torch.randn(nb, hkv, d, bs, device=DEV, dtype=torch.bfloat16)
perm = torch.randperm(nb)
rows_bt = []
o = 0
for p in pers:
    rows_bt.append(perm[o:o + p])
    o += p
q = torch.randn(B, (hq + 2 * hkv) * d, device=DEV, dtype=torch.bfloat16)
ws = ops.decode_workspace(B, hq, d, device=DEV)
out = torch.empty(B, hq * d, device=DEV, dtype=torch.bfloat16)
kv_bytes = sum(lens_list) * hkv * d * 2 * 2

srt = sorted(range(B), key=lambda i: -lens_list[i])
orders = {
    "random": torch.randperm(B, generator=g).tolist(),
    "paired": [srt[z] for z in range(B // 2)] + [srt[B - 1 - z] for z in range(B // 2)],
    "longest_first": srt,
    "shortest_first": srt[::-1],
}
inputs = {}
for name, od in orders.items():
    bt = torch.zeros(B, mb, dtype=torch.int32)
    for z, i in enumerate(od):
        bt[z, :pers[i]] = rows_bt[i]
    lens = torch.tensor([lens_list[i] for i in od], dtype=torch.int32)
    inputs[name] = (bt.to(DEV), lens.to(DEV))

# the engine's fused form (qkv split-K slab reduce + RoPE + cache write of the new token in the
# prologue): 2 slabs, positions = context - 1, no cache write (slot -1)
ncol = (hq + 2 * hkv) * d
slabs = torch.randn(2 * B * ncol, device=DEV, dtype=torch.float32)
cs = torch.randn(maxlen, d, device=DEV, dtype=torch.float32)
slots = torch.full((B,), -1, dtype=torch.int32, device=DEV)
fused_inputs = {k + "_fused": v for k, v in inputs.items() if k in ("random", "paired")}


def run(name, bt, lens):
    if name.endswith("_fused"):
        ops.paged_decode_fused(slabs, 2, lens - 1, cs, slots, kc, vc, bt, lens, hq, hkv, d, 1 / math.sqrt(d),
                               workspace=ws, out=out, splits=1)
    else:
        ops.paged_decode(q, kc, vc, bt, lens, hq, hkv, d, 1 / math.sqrt(d), workspace=ws, out=out, splits=1)


res = {}
for rnd in range(6):
    for name, (bt, lens) in {**inputs, **fused_inputs}.items():
        for _ in range(3):
            run(name, bt, lens)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(True), torch.cuda.Event(True)
        e0.record()
        n = 30
        for _ in range(n):
            run(name, bt, lens)
        e1.record()
        torch.cuda.synchronize()
        res.setdefault(name, []).append(e0.elapsed_time(e1) / n * 1e3)
for name, ts in res.items():
    t = min(ts)
    print(json.dumps({"order": name, "us": round(t, 2), "us_all": [round(x, 1) for x in ts],
                      "TBps": round(kv_bytes / t / 1e6, 2), "ctx_mean": sum(lens_list) / B,
                      "ctx_min": min(lens_list), "ctx_max": max(lens_list)}), flush=True)
