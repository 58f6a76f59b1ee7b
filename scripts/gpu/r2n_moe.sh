# grouped MoE expert GEMM: numerics (ops + Mixtral model), speed vs the per-expert hipBLASLt loop
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_moe_gpu.py -x -v --timeout 120 --timeout-method thread > gpurun_out/moe_tests.log 2>&1 || { tail -40 gpurun_out/moe_tests.log; exit 1; }
tail -3 gpurun_out/moe_tests.log
timeout -k 10 300 python tools/bench_moe_prefill.py > gpurun_out/moe_bench.jsonl 2>gpurun_out/moe_bench.err || { tail gpurun_out/moe_bench.err; exit 1; }
timeout -k 10 300 python tools/bench_moe_prefill.py --tokens 2048 >> gpurun_out/moe_bench.jsonl 2>>gpurun_out/moe_bench.err || exit 1
cat gpurun_out/moe_bench.jsonl
