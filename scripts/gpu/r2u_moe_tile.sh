# MoE prefill with the 256x256 tile kernel behind the grouped path: numerics, MLP microbench,
# then Mixtral-8x7B end to end, grouped (zero host syncs) vs the per-expert loop
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_moe_gpu.py tests/test_gemm_tile_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/moe_tests.log 2>&1 || { tail -40 gpurun_out/moe_tests.log; exit 1; }
tail -2 gpurun_out/moe_tests.log
timeout -k 10 300 python tools/bench_moe_prefill.py > gpurun_out/moe_bench.jsonl 2>gpurun_out/moe_bench.err || { tail gpurun_out/moe_bench.err; exit 1; }
timeout -k 10 300 python tools/bench_moe_prefill.py --tokens 2048 >> gpurun_out/moe_bench.jsonl 2>>gpurun_out/moe_bench.err || exit 1
cat gpurun_out/moe_bench.jsonl
K8SLLM_MOE_PREFILL=grouped timeout -k 10 400 python bench.py --model mixtral-8x7b --steps 2 --warmup 1 > gpurun_out/bmix_grouped.log 2>&1 || { tail -20 gpurun_out/bmix_grouped.log; exit 1; }
tail -1 gpurun_out/bmix_grouped.log | cut -c1-400
K8SLLM_MOE_PREFILL=loop timeout -k 10 400 python bench.py --model mixtral-8x7b --steps 2 --warmup 1 > gpurun_out/bmix_loop.log 2>&1 || { tail -20 gpurun_out/bmix_loop.log; exit 1; }
tail -1 gpurun_out/bmix_loop.log | cut -c1-400
