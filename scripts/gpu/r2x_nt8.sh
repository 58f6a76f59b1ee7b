# experimental 128-column (NT=8) row-major skinny workgroups: correctness, then split sweep vs NT=4
set -o pipefail
mkdir -p gpurun_out
K8SLLM_SKINNY_NT8=1 timeout -k 10 120 python - <<'PY' || exit 1
import torch
from k8s_llm_monitor_amd import ops
torch.manual_seed(0)
for M, N, K, S in ((64, 6144, 4096, 2), (64, 4096, 14336, 4), (5, 4096, 4096, 8), (33, 1024, 1024, 1)):
    a = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
    w = torch.randn(N, K, device="cuda", dtype=torch.bfloat16) * 0.02
    ws = ops.skinny_workspace(M, N, 16, "cuda")
    ns = ops.skinny_slabs(ops.pack_activation(a), w, ws, S, rows=M)
    y = ops.reduce_slabs(ws, ns, M, N).float()
    r = torch.nn.functional.linear(a.float(), w.float())
    err = (y - r).abs().max().item()
    print("nt8 check", M, N, K, S, "max err", round(err, 4))
    assert err < 0.05
PY
timeout -k 10 200 python tools/bench_skinny_rm_splits.py > gpurun_out/nt4.jsonl 2>gpurun_out/nt.err || { tail gpurun_out/nt.err; exit 1; }
K8SLLM_SKINNY_NT8=1 timeout -k 10 200 python tools/bench_skinny_rm_splits.py > gpurun_out/nt8.jsonl 2>>gpurun_out/nt.err || { tail gpurun_out/nt.err; exit 1; }
echo NT4; grep '"waves": 4' gpurun_out/nt4.jsonl; grep '"waves": 2' gpurun_out/nt4.jsonl
echo NT8; grep '"waves": 2' gpurun_out/nt8.jsonl
