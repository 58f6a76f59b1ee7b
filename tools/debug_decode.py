"""Diagnose paged_decode mismatches: per (row, head) max error for several shapes."""
import math, torch
from k8s_llm_monitor_amd import ops
from k8s_llm_monitor_amd.ops import reference as ref
torch.manual_seed(0)
DEV = "cuda"
def run(B, hq, hkv, d, lens_list):
    bs = 16
    maxlen = max(lens_list)
    mb = (maxlen + bs - 1) // bs + 1
    nb = B * mb + 4
    kc = torch.randn(nb, hkv, d // 8, bs, 8, device=DEV, dtype=torch.bfloat16)
    vc = torch.randn(nb, hkv, d, bs, device=DEV, dtype=torch.bfloat16)
    lens = torch.tensor(lens_list, dtype=torch.int32)
    perm = torch.randperm(nb)[: B * mb].view(B, mb).to(torch.int32)
    q = torch.randn(B, hq * d, device=DEV, dtype=torch.bfloat16)
    y = ops.paged_decode(q, kc, vc, perm.to(DEV), lens.to(DEV), hq, hkv, d, 1 / math.sqrt(d))
    r = ref.paged_decode(q.cpu(), kc.cpu(), vc.cpu(), perm, lens, hq, hkv, d, 1 / math.sqrt(d))
    err = (y.cpu().float() - r.float()).abs().view(B, hq, d)
    print(f"B={B} hq={hq} hkv={hkv} lens={lens_list}: max err {err.max():.4f}")
    for b in range(B):
        he = err[b].amax(-1)
        print("  row", b, "len", lens_list[b], "head errs", [round(float(v), 3) for v in he[:8]], "...",
              "dim errs (head0)", [round(float(v), 3) for v in err[b, 0, ::16]])
torch.cuda.synchronize()
run(1, 8, 8, 128, [64])
run(1, 8, 8, 128, [65])
run(1, 8, 8, 128, [128])
run(1, 8, 8, 128, [256])
run(1, 8, 8, 128, [257])
run(1, 32, 8, 128, [200])
run(1, 32, 8, 128, [600])
run(2, 32, 8, 128, [1100, 300])
