# 256x256 MFMA prefill GEMM: numerics, then microbench against hipBLASLt / moe_gemm128
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 240 python -u -m pytest tests/test_gemm_tile_gpu.py -x -v --timeout 120 --timeout-method thread > gpurun_out/gt_tests.log 2>&1 || { tail -40 gpurun_out/gt_tests.log; exit 1; }
tail -3 gpurun_out/gt_tests.log
timeout -k 10 400 python -u tools/bench_gemm_tile.py > gpurun_out/gt_bench.jsonl 2> gpurun_out/gt_bench.err || { tail -20 gpurun_out/gt_bench.err; exit 1; }
cat gpurun_out/gt_bench.jsonl
