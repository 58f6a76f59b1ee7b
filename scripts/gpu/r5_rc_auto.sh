# the row-complete o projection on by default for the smallest decode buckets: kernel parity,
# the per-bucket A/B that picks RC_O_MAX_ROWS, batch-1 latency and the headline with the default
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_gemm_decode_gpu.py tests/test_decode_fusion.py tests/test_real_shape_gpu.py > gpurun_out/rca_tests.log 2>&1
echo "tests rc=$?"; tail -2 gpurun_out/rca_tests.log
timeout -k 10 400 python -u tools/bench_decode_step.py --switch rc --rows 1,2,4,8,16,32 --rounds 2 --tokens 64 \
  > gpurun_out/rca_rows.jsonl 2> gpurun_out/rca_rows.err || { tail -20 gpurun_out/rca_rows.err; exit 1; }
grep on_median gpurun_out/rca_rows.jsonl
timeout -k 10 300 python bench.py --mode latency --steps 5 --warmup 1 --out gpurun_out/rca_lat.json \
  > gpurun_out/rca_lat.log 2>&1 || { tail -20 gpurun_out/rca_lat.log; exit 1; }
python3 -c "import json;a=json.load(open('gpurun_out/rca_lat.json'));print('lat', a['p50_latency_ms'], a['tpot_ms'])"
timeout -k 10 400 python bench.py --out gpurun_out/rca_bench.json > gpurun_out/rca_bench.log 2>&1 || { tail -20 gpurun_out/rca_bench.log; exit 1; }
tail -c 400 gpurun_out/rca_bench.json
