# Llama-3-70B TP=1 on one GPU with the final tree (single weight copy, burst-aware mixing)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python bench.py --model llama-3-70b --steps 1 --warmup 1 --kv-cache-gb 60 > gpurun_out/b70f.log 2>&1 || { tail -20 gpurun_out/b70f.log; exit 1; }
tail -1 gpurun_out/b70f.log | cut -c1-300
