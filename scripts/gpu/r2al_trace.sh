# wave-boundary timeline of the headline (engine trace)
set -o pipefail
mkdir -p gpurun_out
K8SLLM_TRACE=1 timeout -k 10 300 python bench.py --steps 4 --warmup 1 > gpurun_out/trace_b.log 2>&1 || { tail -20 gpurun_out/trace_b.log; exit 1; }
grep "\[trace\]" gpurun_out/trace_b.log | head -40
tail -1 gpurun_out/trace_b.log | cut -c60-140
