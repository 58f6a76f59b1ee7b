# the driver's multi-GPU launch form rehearsed on the one GPU: torchrun, 2 ranks, the real
# Llama-3-8B headline bench (both ranks on cuda:0, gloo process groups: RCCL refuses two ranks on
# one device) - exercises the launch, barriers, max-over-ranks timing and the JSON line
set -o pipefail
mkdir -p gpurun_out
export K8SLLM_DEVICE=cuda:0 K8SLLM_DIST_BACKEND=gloo
timeout -k 10 900 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29533 bench.py --gpus 2 --steps 2 --warmup 1 --kv-cache-gb 24 --out gpurun_out/dp2_torchrun.json \
  > gpurun_out/dp2_torchrun.log 2>&1 || { grep -v Gloo gpurun_out/dp2_torchrun.log | tail -30; exit 1; }
cut -c1-700 gpurun_out/dp2_torchrun.json
