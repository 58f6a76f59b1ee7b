# Llama-3-70B and Mixtral-8x7B on ONE GPU with the single resident weight copy (skinny decode path)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python bench.py --model llama-3-70b --steps 1 --warmup 1 --kv-cache-gb 60 > gpurun_out/b70.log 2>&1 || { tail -20 gpurun_out/b70.log; exit 1; }
tail -1 gpurun_out/b70.log
timeout -k 10 400 python bench.py --model mixtral-8x7b --steps 2 --warmup 1 > gpurun_out/bmix.log 2>&1 || { tail -20 gpurun_out/bmix.log; exit 1; }
tail -1 gpurun_out/bmix.log
