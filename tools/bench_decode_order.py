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

res = {}
for rnd in range(6):
    for name, (bt, lens) in inputs.items():
        for _ in range(3):
            ops.paged_decode(q, kc, vc, bt, lens, hq, hkv, d, 1 / math.sqrt(d), workspace=ws, out=out, splits=1)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(True), torch.cuda.Event(True)
        e0.record()
        n = 30
        for _ in range(n):
            ops.paged_decode(q, kc, vc, bt, lens, hq, hkv, d, 1 / math.sqrt(d), workspace=ws, out=out, splits=1)
        e1.record()
        torch.cuda.synchronize()
        res.setdefault(name, []).append(e0.elapsed_time(e1) / n * 1e3)
for name, ts in res.items():
    t = min(ts)
    print(json.dumps({"order": name, "us": round(t, 2), "us_all": [round(x, 1) for x in ts],
                      "TBps": round(kv_bytes / t / 1e6, 2), "ctx_mean": sum(lens_list) / B,
                      "ctx_min": min(lens_list), "ctx_max": max(lens_list)}), flush=True)
