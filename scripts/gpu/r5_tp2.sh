# TP=2 on the one GPU after capping the IPC all-reduce grid: serial and overlapped engine
# rehearsals, then the overlap timeline tool with per-rank kernel traces.
set -o pipefail
mkdir -p gpurun_out
fatal() { case $1 in 124|134|137|139) echo "fatal rc $1"; exit 1;; esac; }
timeout -k 10 700 python -u -m pytest tests/test_gemm_decode_gpu.py tests/test_tile_real_shapes_gpu.py \
  tests/test_real_shape_gpu.py "tests/test_ops_gpu.py::test_flash_prefill_paged_v2_long_prompts" \
  "tests/test_ops_gpu.py::test_flash_prefill_paged_v2_moderate_max_jumps" -m gpu -q --timeout 300 \
  --timeout-method thread > gpurun_out/r5_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "passed|failed|FAILED" gpurun_out/r5_tests.log | tail -12; fatal $rc
K8SLLM_TP_OVERLAP=0 bash scripts/gpu/run.sh rehearse tp2serial --gpus 2 --tp 2 --model llama-tiny-d128 --steps 2 --warmup 1
rc=$?; echo "rehearsal serial rc=$rc"; fatal $rc
bash scripts/gpu/run.sh rehearse tp2ov --gpus 2 --tp 2 --model llama-tiny-d128 --steps 2 --warmup 1
rc=$?; echo "rehearsal overlap rc=$rc"; fatal $rc
root=$PWD; cd /tmp && export TMPDIR=/tmp && cd "$root"
timeout -k 10 400 python tools/tp_overlap_timeline.py --world 2 --model llama-3-8b --layers 8 --seqs 4 --len 512 \
  --prof gpurun_out/ovl > gpurun_out/ovl_run.jsonl 2> gpurun_out/ovl_run.err
rc=$?; echo "timeline rc=$rc"; grep -v Gloo gpurun_out/ovl_run.jsonl; fatal $rc
[ $rc = 0 ] || { grep -v "Gloo\|socket" gpurun_out/ovl_run.err | tail -20; exit 1; }
python tools/tp_overlap_timeline.py --analyze gpurun_out/ovl | tee gpurun_out/ovl_analyze.jsonl
find gpurun_out/ovl -name "*results.db" -size +30M -delete
