# paged decode with one 16-byte V load per lane and dim tile: parity tests, in-engine kernel trace, headline
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests/test_ops_gpu.py tests/test_real_shape_gpu.py tests/test_tp_gpu.py tests/test_engine.py -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/dec_tests.log 2>&1 || { tail -40 gpurun_out/dec_tests.log; exit 1; }
tail -1 gpurun_out/dec_tests.log
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/pt_dec -o run -- python3 bench.py --steps 1 --warmup 1 > gpurun_out/pt_dec.log 2>&1 || { tail -30 gpurun_out/pt_dec.log; exit 1; }
f=$(find gpurun_out/pt_dec -name "*results.db" | head -1)
python3 - "$f" > gpurun_out/dec_trace.txt <<'PY'
import sqlite3, sys, collections
c = sqlite3.connect(sys.argv[1])
agg = collections.defaultdict(list)
for name, s, e in c.execute("select name, start, end from kernels"):
    for k in ("paged_decode_kernel<128, 4, true, 32>", "paged_decode_kernel<128, 4, true, 64>", "gemm_skinny_rm_kernel<4, 4, 3, 2", "add_norm_partial"):
        if k in name:
            agg[k].append(e - s)
print(" | ".join(f"{k}: {sum(v)/len(v)/1e3:.2f} us x{len(v)}" for k, v in agg.items()))
PY
cat gpurun_out/dec_trace.txt
rm -rf gpurun_out/pt_dec
timeout -k 10 300 python bench.py --steps 5 --warmup 2 --out gpurun_out/bench_dec.json > gpurun_out/bench_dec.log 2>&1 || { tail -20 gpurun_out/bench_dec.log; exit 1; }
cut -c1-200 gpurun_out/bench_dec.json
timeout -k 10 200 python bench.py --mode latency --steps 3 --warmup 1 --out gpurun_out/lat_dec.json > gpurun_out/lat_dec.log 2>&1 || { tail -20 gpurun_out/lat_dec.log; exit 1; }
cut -c1-200 gpurun_out/lat_dec.json
