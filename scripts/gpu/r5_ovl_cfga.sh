# TP=2 overlap timeline on the one GPU (the tool now stages the q-block schedule like the runner:
# no host copies in the step), at 2048 and 4096 tokens; then BASELINE configs 4 / 5 (part a)
set -o pipefail
mkdir -p gpurun_out
root=$PWD; cd /tmp && export TMPDIR=/tmp && cd "$root"
for sl in 4:512 4:1024; do
  tag=ovl_${sl%%:*}x${sl##*:}
  timeout -k 10 400 python tools/tp_overlap_timeline.py --world 2 --model llama-3-8b --layers 8 --seqs ${sl%%:*} \
    --len ${sl##*:} --prof gpurun_out/$tag > gpurun_out/${tag}_run.jsonl 2> gpurun_out/${tag}_run.err \
    || { grep -v "Gloo\|socket" gpurun_out/${tag}_run.err | tail -20; exit 1; }
  grep -v Gloo gpurun_out/${tag}_run.jsonl | cut -c1-330
  python tools/tp_overlap_timeline.py --analyze gpurun_out/$tag > gpurun_out/${tag}_analyze.jsonl
  cut -c1-400 gpurun_out/${tag}_analyze.jsonl
done
bash scripts/gpu/r5_configs.sh a
