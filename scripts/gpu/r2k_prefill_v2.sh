# flash prefill v2 (paged, LDS-DMA tiles, GQA-shared) + V-cache token permutation: numerics, microbench
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_ops_gpu.py -x -q -k "prefill" --timeout 120 --timeout-method thread > gpurun_out/pf2_tests.log 2>&1 || { tail -40 gpurun_out/pf2_tests.log; exit 1; }
tail -2 gpurun_out/pf2_tests.log
timeout -k 10 200 python tools/bench_prefill_attn.py > gpurun_out/pf2_bench.jsonl 2>gpurun_out/pf2_bench.err || { tail gpurun_out/pf2_bench.err; exit 1; }
timeout -k 10 200 python tools/bench_prefill_attn.py --seqs 4 --len 4000 >> gpurun_out/pf2_bench.jsonl 2>>gpurun_out/pf2_bench.err || { tail gpurun_out/pf2_bench.err; exit 1; }
cat gpurun_out/pf2_bench.jsonl
