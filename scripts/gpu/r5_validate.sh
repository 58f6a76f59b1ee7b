# tree validation after the round-5 commit: GPU suite + smoke + headline, then a one-GPU TP=2
# rehearsal (exercises the micro-batched prefill overlap through the engine)
set -o pipefail
mkdir -p gpurun_out
bash scripts/gpu/run.sh suite || exit 1
bash scripts/gpu/run.sh rehearse tp2ov --gpus 2 --tp 2 --model llama-tiny-d128 --steps 2 --warmup 1 || exit 1
