# full GPU suite, smoke, headline bench, and the TP=2 bench path on one GPU (tiny model)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/gputests.log 2>&1 || { tail -40 gpurun_out/gputests.log; exit 1; }
tail -2 gpurun_out/gputests.log
timeout -k 10 300 python -u __graft_entry__.py smoke > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 300 python bench.py --steps 5 --warmup 2 > gpurun_out/bench_w.log 2>&1 || { tail -20 gpurun_out/bench_w.log; exit 1; }
tail -1 gpurun_out/bench_w.log | cut -c1-300
export K8SLLM_DEVICE=cuda:0 K8SLLM_DIST_BACKEND=gloo
timeout -k 10 170 python -u bench.py --gpus 2 --tp 2 --model llama-tiny-d128 --batch 8 --max-new-tokens 32 --steps 2 --warmup 1 --kv-cache-gb 4 > gpurun_out/rh_tp2_tiny.log 2>&1 || { grep -v Gloo gpurun_out/rh_tp2_tiny.log | tail -20; exit 1; }
tail -1 gpurun_out/rh_tp2_tiny.log | cut -c1-400
