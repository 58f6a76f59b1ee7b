# qkv projection + fused RoPE epilogue on gemm_tile: numerics, then headline A/B against the
# library qkv + rope_cache pass (K8SLLM_QKV_ROPE_TILE=0) and all-tile routing, interleaved processes
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_tile_real_shapes_gpu.py tests/test_moe_gpu.py tests/test_gemm_tile_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/t_rope.log 2>&1 || { tail -30 gpurun_out/t_rope.log; exit 1; }
tail -1 gpurun_out/t_rope.log
for r in 1 2; do
  for v in rope norope alltile; do
    case $v in
      rope) env_="K8SLLM_QKV_ROPE_TILE=1 K8SLLM_PREFILL_GEMM=auto";;
      norope) env_="K8SLLM_QKV_ROPE_TILE=0 K8SLLM_PREFILL_GEMM=auto";;
      alltile) env_="K8SLLM_QKV_ROPE_TILE=1 K8SLLM_PREFILL_GEMM=tile";;
    esac
    export $env_
    timeout -k 10 300 python bench.py --steps 4 --warmup 2 --out gpurun_out/bench_rope_${v}_$r.json > gpurun_out/bench_rope_${v}_$r.log 2>&1 || { tail -20 gpurun_out/bench_rope_${v}_$r.log; exit 1; }
    echo "$v $r $(cut -c1-120 gpurun_out/bench_rope_${v}_$r.json)"
  done
done
