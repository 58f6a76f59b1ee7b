# row-major LDS-DMA skinny GEMM: numerics, then packed vs row-major timing
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_skinny_rm_gpu.py -x -v --timeout 120 --timeout-method thread > gpurun_out/rm_tests.log 2>&1 || { tail -40 gpurun_out/rm_tests.log; exit 1; }
tail -3 gpurun_out/rm_tests.log
timeout -k 10 300 python -u tools/bench_skinny_rm.py > gpurun_out/rm_bench.jsonl 2> gpurun_out/rm_bench.err || { tail -20 gpurun_out/rm_bench.err; exit 1; }
cat gpurun_out/rm_bench.jsonl
