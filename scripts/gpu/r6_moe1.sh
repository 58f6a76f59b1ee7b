# round 6: ONE_LAYOUT for MoE (packed attention projections and experts only) - the MoE / engine /
# TP / real-shape GPU tests, then Mixtral-8x7B TP=1 headline one vs two layouts
set -o pipefail
mkdir -p gpurun_out
bash scripts/gpu/run.sh tests 'moe or mixtral or engine or tp or one_layout or real_shape or checkpoint' || exit 1
timeout -k 10 600 python bench.py --model mixtral-8x7b --steps 3 --warmup 1 --layout one --out gpurun_out/mx_one.json \
  > gpurun_out/mx_one.log 2>&1 || { tail -20 gpurun_out/mx_one.log; exit 1; }
cut -c1-200 gpurun_out/mx_one.json
timeout -k 10 600 python bench.py --model mixtral-8x7b --steps 3 --warmup 1 --layout two --out gpurun_out/mx_two.json \
  > gpurun_out/mx_two.log 2>&1 || { tail -20 gpurun_out/mx_two.log; exit 1; }
cut -c1-200 gpurun_out/mx_two.json
