# headline A/B: every prefill projection on gemm_tile vs the default routing (hipBLASLt for
# qkv / o / down), interleaved processes; plus the per-shape GEMM microbench
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_moe_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/t_moe.log 2>&1 || { tail -30 gpurun_out/t_moe.log; exit 1; }
tail -1 gpurun_out/t_moe.log
timeout -k 10 400 python tools/bench_gemm_tile.py --only qkv,o,down --impl w4s,hipblaslt > gpurun_out/gemm_r4.jsonl 2> gpurun_out/gemm_r4.err || { tail -20 gpurun_out/gemm_r4.err; exit 1; }
cat gpurun_out/gemm_r4.jsonl
for r in 1 2; do
  for mode in auto tile; do
    K8SLLM_PREFILL_GEMM=$mode timeout -k 10 300 python bench.py --steps 4 --warmup 2 --out gpurun_out/bench_pg_${mode}_$r.json > gpurun_out/bench_pg_${mode}_$r.log 2>&1 || { tail -20 gpurun_out/bench_pg_${mode}_$r.log; exit 1; }
    echo "$mode $r $(cut -c1-120 gpurun_out/bench_pg_${mode}_$r.json)"
  done
done
