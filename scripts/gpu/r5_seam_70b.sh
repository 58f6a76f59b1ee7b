# the new GPU TP overlap test, the seam-fusion A/B (ring filled before the norm phase), and the
# Llama-3-70B TP=1 proxy of config 4
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_tp_gpu.py -m gpu -q -k overlap --timeout 240 --timeout-method thread \
  > gpurun_out/t_ovl.log 2>&1 || { tail -30 gpurun_out/t_ovl.log; exit 1; }
tail -1 gpurun_out/t_ovl.log
bash scripts/gpu/r5_seam.sh || exit 1
bash scripts/gpu/r5_configs.sh c
