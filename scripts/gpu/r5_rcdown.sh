# row-complete down projection (K = 14336) in the small decode buckets: parity, the real-shape
# engine tests, then decode-step A/B at 1 / 4 / 16 / 32 rows
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_gemm_decode_gpu.py -k rc_down -m gpu \
  > gpurun_out/rd_tests.log 2>&1
echo "tests rc=$?"; tail -3 gpurun_out/rd_tests.log
grep -q " passed" gpurun_out/rd_tests.log && ! grep -q "failed\|error" gpurun_out/rd_tests.log || exit 1
timeout -k 10 400 python -u tools/bench_decode_step.py --switch rc_down --rows 1,4,16 --rounds 3 --tokens 64 \
  > gpurun_out/rd_ab.jsonl 2> gpurun_out/rd_ab.err || { tail -20 gpurun_out/rd_ab.err; exit 1; }
grep on_median gpurun_out/rd_ab.jsonl
