"""Microbenchmark of paged_decode at serving shapes: sweep the split count in one process."""
import math
import sys

import torch

from k8s_llm_monitor_amd import ops

torch.manual_seed(0)
DEV = "cuda"
hq, hkv, d, bs = 32, 8, 128, 16
B = int(sys.argv[1]) if len(sys.argv) > 1 else 64
ctx = int(sys.argv[2]) if len(sys.argv) > 2 else 1800
maxlen = 8192
mb = maxlen // bs
per = ctx // bs + 2
nb = B * per + 8
kc = torch.randn(nb, hkv, d // 8, bs, 8, device=DEV, dtype=torch.bfloat16)
vc = torch.randn(nb, hkv, d, bs, device=DEV, dtype=torch.bfloat16)
perm = torch.randperm(nb, device=DEV)[: B * per].view(B, per).to(torch.int32)
bt = torch.zeros(B, mb, dtype=torch.int32, device=DEV)
bt[:, :per] = perm
lens = torch.full((B,), ctx, dtype=torch.int32, device=DEV)
q = torch.randn(B, (hq + 2 * hkv) * d, device=DEV, dtype=torch.bfloat16)
ws = ops.decode_workspace(B, hq, d, device=DEV)
out = torch.empty(B, hq * d, device=DEV, dtype=torch.bfloat16)
kv_bytes = B * ctx * hkv * d * 2 * 2
res = {}
cands = [1, 2, 4, 8, 16, 32]
for rnd in range(5):
    for S in cands:
        for _ in range(2):
            ops.paged_decode(q, kc, vc, bt, lens, hq, hkv, d, 1 / math.sqrt(d), workspace=ws, out=out, splits=S)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(True), torch.cuda.Event(True)
        e0.record()
        n = 20
        for _ in range(n):
            ops.paged_decode(q, kc, vc, bt, lens, hq, hkv, d, 1 / math.sqrt(d), workspace=ws, out=out, splits=S)
        e1.record()
        torch.cuda.synchronize()
        res.setdefault(S, []).append(e0.elapsed_time(e1) / n * 1e3)
auto = ops.decode_splits(B, hkv)
for S, ts in res.items():
    t = min(ts)
    print(f"B={B} ctx={ctx} S={S:2d}{' (auto)' if S == auto else '       '} best {t:7.1f} us  "
          f"{kv_bytes / t / 1e6:.2f} TB/s")
