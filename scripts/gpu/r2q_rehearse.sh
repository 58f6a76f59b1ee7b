# multi-rank launch rehearsals on the one-GPU box: bench.py spawns 2 rank processes itself
# (DP=2 and TP=2; every rank pinned to cuda:0, gloo process group: RCCL refuses 2 ranks/device)
set -o pipefail
mkdir -p gpurun_out
export K8SLLM_DEVICE=cuda:0 K8SLLM_DIST_BACKEND=gloo
timeout -k 10 500 python bench.py --gpus 2 --steps 2 --warmup 1 --kv-cache-gb 24 > gpurun_out/rh_dp2.log 2>&1 || { tail -30 gpurun_out/rh_dp2.log; exit 1; }
tail -1 gpurun_out/rh_dp2.log
timeout -k 10 500 python bench.py --gpus 2 --tp 2 --steps 2 --warmup 1 --kv-cache-gb 24 > gpurun_out/rh_tp2.log 2>&1 || { tail -30 gpurun_out/rh_tp2.log; exit 1; }
tail -1 gpurun_out/rh_tp2.log
