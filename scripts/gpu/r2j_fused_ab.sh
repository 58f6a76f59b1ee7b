# in-launch fused epilogues (RESNORM o/down, ROPE qkv) on the row-major kernel vs slab + reduce kernels
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_skinny_rm_gpu.py tests/test_ops_gpu.py -x -q -k "resnorm or rope or rm_" --timeout 120 --timeout-method thread > gpurun_out/fused_tests.log 2>&1 || { tail -30 gpurun_out/fused_tests.log; exit 1; }
tail -1 gpurun_out/fused_tests.log
for f in 0 1 0 1; do
K8SLLM_FUSED_EPI=$f timeout -k 10 300 python bench.py --steps 4 --warmup 2 > gpurun_out/bench_fused$f.log 2>&1 || { tail -20 gpurun_out/bench_fused$f.log; exit 1; }
echo "FUSED_EPI=$f $(tail -1 gpurun_out/bench_fused$f.log | cut -c1-200)"
done
