# end-of-round validation of the committed tree: GPU suite + smoke + headline, then the driver's
# multi-rank launch form (torchrun, DP=2 on the one GPU) and a TP=2 rehearsal
set -o pipefail
mkdir -p gpurun_out
bash scripts/gpu/run.sh suite || exit 1
bash scripts/gpu/r5_dp2_torchrun.sh || exit 1
bash scripts/gpu/run.sh rehearse tp2final --gpus 2 --tp 2 --model llama-tiny-d128 --steps 2 --warmup 1 || exit 1
