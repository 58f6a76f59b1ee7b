# in-engine A/B of the DMA/MFMA interleave and the one-round-trip add_norm_partial: kernel traces
# of the headline with the new forms vs K8SLLM_SKINNY_ILV=0 K8SLLM_ANP_STATIC=0, same box, alternating
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
: > gpurun_out/ilv_trace_ab.txt
for r in 1 2; do for v in 1 0; do
  K8SLLM_SKINNY_ILV=$v K8SLLM_ANP_STATIC=$v timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/pt_$v -o run -- python3 bench.py --steps 1 --warmup 1 > gpurun_out/pt_$v.log 2>&1 || { tail -30 gpurun_out/pt_$v.log; exit 1; }
  f=$(find gpurun_out/pt_$v -name "*results.db" | head -1)
  python3 - "$f" "$v" "$r" >> gpurun_out/ilv_trace_ab.txt <<'PY'
import sqlite3, sys, collections
c = sqlite3.connect(sys.argv[1])
agg = collections.defaultdict(list)
for name, s, e in c.execute("select name, start, end from kernels"):
    for k in ("gemm_skinny_rm_kernel<4, 4, 3, 2", "gemm_skinny_rm_kernel<4, 4, 0, 4", "gemm_skinny_rm_kernel<4, 3, 0, 4", "add_norm_partial", "paged_decode_kernel<128, 4, true, 32>"):
        if k in name:
            agg[k].append(e - s)
print(f"new={sys.argv[2]} round={sys.argv[3]} " + " | ".join(f"{k}: {sum(v)/len(v)/1e3:.2f} us x{len(v)}" for k, v in agg.items()))
PY
  rm -rf gpurun_out/pt_$v
done; done
cat gpurun_out/ilv_trace_ab.txt
