# secondary BASELINE configs with the current tree: pod-communication path (config 3), Mixtral (5), batch-1 latency
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --path podcomm --steps 3 --warmup 1 > gpurun_out/podcomm.log 2>&1 || { tail -20 gpurun_out/podcomm.log; exit 1; }
tail -1 gpurun_out/podcomm.log | cut -c1-250
timeout -k 10 400 python bench.py --model mixtral-8x7b --steps 2 --warmup 1 > gpurun_out/bmix2.log 2>&1 || { tail -20 gpurun_out/bmix2.log; exit 1; }
tail -1 gpurun_out/bmix2.log | cut -c1-250
timeout -k 10 300 python bench.py --mode latency --batch 1 --steps 8 --warmup 2 > gpurun_out/lat1.log 2>&1 || { tail -20 gpurun_out/lat1.log; exit 1; }
tail -1 gpurun_out/lat1.log | cut -c1-250
