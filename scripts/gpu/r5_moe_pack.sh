# MoE decode: the normed rows' packed copy written by reduce_add_rmsnorm (no torch pack pass):
# MoE / engine GPU tests, then the Mixtral bench (config 5)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread \
  tests/test_moe_gpu.py tests/test_engine.py tests/test_ops_gpu.py -m gpu -k "moe or norm or decode" \
  > gpurun_out/mp_tests.log 2>&1
echo "tests rc=$?"; tail -2 gpurun_out/mp_tests.log
grep -q " passed" gpurun_out/mp_tests.log && ! grep -q "failed\|error" gpurun_out/mp_tests.log || exit 1
timeout -k 10 700 python bench.py --model mixtral-8x7b --steps 3 --warmup 1 --out gpurun_out/mp_mixtral.json \
  > gpurun_out/mp_mixtral.log 2>&1 || { tail -20 gpurun_out/mp_mixtral.log; exit 1; }
cut -c1-300 gpurun_out/mp_mixtral.json
