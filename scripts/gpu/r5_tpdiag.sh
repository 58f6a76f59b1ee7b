# TP=2 on the one GPU: (1) the serial-all-reduce rehearsal (K8SLLM_TP_OVERLAP=0), (2) the
# overlapped-prefill timeline tool (8B shapes, 8 layers, IPC all-reduce on the comm stream) with
# per-rank kernel traces.  A Python-level failure of (1) still runs (2); a fault / abort / time
# limit ends the script.
set -o pipefail
mkdir -p gpurun_out
fatal() { case $1 in 124|134|137|139) echo "fatal rc $1"; exit 1;; esac; }
K8SLLM_TP_OVERLAP=0 bash scripts/gpu/run.sh rehearse tp2serial --gpus 2 --tp 2 --model llama-tiny-d128 --steps 2 --warmup 1
rc=$?; echo "rehearsal serial rc=$rc"; fatal $rc
root=$PWD; cd /tmp && export TMPDIR=/tmp && cd "$root"
timeout -k 10 400 python tools/tp_overlap_timeline.py --world 2 --model llama-3-8b --layers 8 --seqs 4 --len 512 \
  --prof gpurun_out/ovl > gpurun_out/ovl_run.jsonl 2> gpurun_out/ovl_run.err
rc=$?; echo "timeline rc=$rc"; grep -v Gloo gpurun_out/ovl_run.jsonl; fatal $rc
[ $rc = 0 ] || { grep -v "Gloo\|socket" gpurun_out/ovl_run.err | tail -20; exit 1; }
python tools/tp_overlap_timeline.py --analyze gpurun_out/ovl | tee gpurun_out/ovl_analyze.jsonl
find gpurun_out/ovl -name "*results.db" -size +30M -delete
