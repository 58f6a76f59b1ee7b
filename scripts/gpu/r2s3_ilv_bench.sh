# headline A/B: interleaved skinny DMA/MFMA (default) vs K8SLLM_SKINNY_ILV=0, alternating; GPU suite first
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gputests.log 2>&1 || { tail -40 gpurun_out/gputests.log; exit 1; }
tail -1 gpurun_out/gputests.log
for r in 1 2; do
  for v in 1 0; do
    K8SLLM_SKINNY_ILV=$v timeout -k 10 300 python bench.py --steps 5 --warmup 2 --out gpurun_out/ilv_bench_${v}_r$r.json > gpurun_out/ilv_bench_${v}_r$r.log 2>&1 || { tail -20 gpurun_out/ilv_bench_${v}_r$r.log; exit 1; }
    echo "ilv=$v r=$r $(cut -c1-170 gpurun_out/ilv_bench_${v}_r$r.json)"
  done
done
