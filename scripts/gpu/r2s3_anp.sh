# add_norm_partial with a compile-time slab count (one memory round trip) vs the runtime-count form
set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/anp.jsonl
for r in 1 2; do for v in 1 0; do
  K8SLLM_ANP_STATIC=$v timeout -k 10 120 python -u tools/bench_add_norm.py 2>/dev/null >> gpurun_out/anp.jsonl || exit 1
done; done
cat gpurun_out/anp.jsonl
timeout -k 10 300 python -u -m pytest tests/test_skinny_rm_gpu.py tests/test_ops_gpu.py tests/test_real_shape_gpu.py -x -q --timeout 240 --timeout-method thread > gpurun_out/anp_tests.log 2>&1 || { tail -30 gpurun_out/anp_tests.log; exit 1; }
tail -1 gpurun_out/anp_tests.log
