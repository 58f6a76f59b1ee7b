# round 6: Llama-3-70B at TP=1 with ONE weight layout - every projection (MLP included) on the
# packed shared-A decode GEMM at no extra memory (MLP >= 5.6 TB/s, step <= 33 ms)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_real_shape_gpu.py -m gpu -q --timeout 300 \
  --timeout-method thread > gpurun_out/t_70b.log 2>&1 || { tail -30 gpurun_out/t_70b.log; exit 1; }
tail -1 gpurun_out/t_70b.log
timeout -k 10 700 python bench.py --model llama-3-70b --steps 2 --warmup 1 --out gpurun_out/cfg_l70_one.json \
  > gpurun_out/cfg_l70_one.log 2>&1 || { tail -20 gpurun_out/cfg_l70_one.log; exit 1; }
cut -c1-300 gpurun_out/cfg_l70_one.json
bash scripts/gpu/run.sh prof l70one --model llama-3-70b > gpurun_out/prof_l70one_out.txt 2>&1 || { tail -20 gpurun_out/prof_l70one_out.txt; exit 1; }
head -3 gpurun_out/prof_l70one_steps.txt; head -14 gpurun_out/prof_l70one_summary.md
