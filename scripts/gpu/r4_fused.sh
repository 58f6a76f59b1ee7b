# prefill RMSNorms folded into the tile GEMM epilogues: numerics, headline A/B (fused vs
# K8SLLM_FUSED_NORM=0, interleaved), production serving with the context-aware admission model
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_tile_real_shapes_gpu.py tests/test_gemm_tile_gpu.py tests/test_real_shape_gpu.py -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/t_fused.log 2>&1 || { tail -40 gpurun_out/t_fused.log; exit 1; }
tail -2 gpurun_out/t_fused.log
for r in 1 2; do
  for v in 1 0; do
    K8SLLM_FUSED_NORM=$v timeout -k 10 300 python bench.py --steps 4 --warmup 2 --out gpurun_out/bench_fn${v}_$r.json > gpurun_out/bench_fn${v}_$r.log 2>&1 || { tail -20 gpurun_out/bench_fn${v}_$r.log; exit 1; }
    echo "fused=$v $r $(cut -c80-110 gpurun_out/bench_fn${v}_$r.json)"
  done
done
timeout -k 10 400 python bench.py --production --max-new-tokens 2000 --steps 2 --warmup 1 --out gpurun_out/prod2000_kv2.json > gpurun_out/prod2000_kv2.log 2>&1 || { tail -20 gpurun_out/prod2000_kv2.log; exit 1; }
python3 -c "import json;d=json.load(open('gpurun_out/prod2000_kv2.json'));print(d['value'], d['requests'], d['tpot_model_ms'].get('kv_fit'), d['ttft_ms'], d['tpot_ms'], d['p99_latency_ms'], d['config']['prompt_tokens_mean'])"
