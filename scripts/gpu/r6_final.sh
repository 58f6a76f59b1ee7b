# round 6 validation of the committed tree, part 1: GPU suite + smoke + headline, smoke's fault
# injection, the driver's torchrun DP=2 launch form and a TP=2 rehearsal on the one GPU
set -o pipefail
mkdir -p gpurun_out
bash scripts/gpu/run.sh suite || exit 1
timeout -k 10 300 python -u tools/smoke_fault.py > gpurun_out/smoke_fault.log 2>&1 || { tail -20 gpurun_out/smoke_fault.log; exit 1; }
tail -1 gpurun_out/smoke_fault.log
bash scripts/gpu/r5_dp2_torchrun.sh || exit 1
bash scripts/gpu/run.sh rehearse tp2final --gpus 2 --tp 2 --model llama-tiny-d128 --steps 2 --warmup 1 || exit 1
