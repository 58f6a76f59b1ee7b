# Llama-3-70B TP=1 with the LM head and attention projections on gemm_decode (MLP stays row-major)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_real_shape_gpu.py tests/test_gemm_decode_gpu.py -m gpu -q --timeout 300 \
  --timeout-method thread > gpurun_out/t_70b.log 2>&1 || { tail -30 gpurun_out/t_70b.log; exit 1; }
tail -1 gpurun_out/t_70b.log
bash scripts/gpu/r5_configs.sh c
bash scripts/gpu/run.sh prof l70 --model llama-3-70b > gpurun_out/prof_l70_out.txt 2>&1 || { tail -20 gpurun_out/prof_l70_out.txt; exit 1; }
head -3 gpurun_out/prof_l70_steps.txt; grep -c "Cijk_" gpurun_out/prof_l70_summary.md || true
