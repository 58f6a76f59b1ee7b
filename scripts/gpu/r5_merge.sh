# in-launch merge of the paged-decode split partials: bit-identity vs the reduce launch, the GPU
# decode suites, then decode-step A/B at the batch sizes that split (1 / 4 / 16 rows)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_ops_gpu.py tests/test_real_shape_gpu.py tests/test_engine.py -k "decode or merge or real_shape" -m gpu \
  > gpurun_out/mg_tests.log 2>&1
echo "tests rc=$?"; tail -3 gpurun_out/mg_tests.log
grep -q " passed" gpurun_out/mg_tests.log && ! grep -q "failed\|error" gpurun_out/mg_tests.log || exit 1
timeout -k 10 400 python -u tools/bench_decode_step.py --switch merge --rows 1,4,16 --rounds 3 --tokens 64 \
  > gpurun_out/mg_ab.jsonl 2> gpurun_out/mg_ab.err || { tail -20 gpurun_out/mg_ab.err; exit 1; }
grep on_median gpurun_out/mg_ab.jsonl
