# q-block LPT order by causal key span (cached prefix + first row): prefill GPU tests, in-engine flash trace, headline
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gputests.log 2>&1 || { tail -40 gpurun_out/gputests.log; exit 1; }
tail -1 gpurun_out/gputests.log
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/pt_lpt -o run -- python3 bench.py --steps 2 --warmup 1 > gpurun_out/pt_lpt.log 2>&1 || { tail -30 gpurun_out/pt_lpt.log; exit 1; }
f=$(find gpurun_out/pt_lpt -name "*results.db" | head -1)
python3 - "$f" > gpurun_out/lpt_trace.txt <<'PY'
import sqlite3, sys, collections
c = sqlite3.connect(sys.argv[1])
agg = collections.defaultdict(list)
for name, s, e in c.execute("select name, start, end from kernels"):
    for k in ("flash_prefill_paged_v2_kernel", "paged_decode_kernel<128, 4, true, 32>", "gemm_skinny_rm_kernel<4, 4, 3, 2"):
        if k in name:
            agg[k].append(e - s)
print(" | ".join(f"{k}: {sum(v)/len(v)/1e3:.2f} us x{len(v)}" for k, v in agg.items()))
PY
cat gpurun_out/lpt_trace.txt
rm -rf gpurun_out/pt_lpt
timeout -k 10 300 python bench.py --steps 5 --warmup 2 --out gpurun_out/bench_lpt.json > gpurun_out/bench_lpt.log 2>&1 || { tail -20 gpurun_out/bench_lpt.log; exit 1; }
cut -c1-160 gpurun_out/bench_lpt.json
