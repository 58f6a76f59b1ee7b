# sampler: vocabulary parts per row (workgroups per row) at the decode batch
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python tools/bench_sampler.py --parts 1,2,4,8,16,32 > gpurun_out/sampler_parts.jsonl 2> gpurun_out/sampler_parts.err || { tail -20 gpurun_out/sampler_parts.err; exit 1; }
cat gpurun_out/sampler_parts.jsonl
