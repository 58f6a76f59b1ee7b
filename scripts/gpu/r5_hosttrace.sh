# host side of the decode pipeline: the headline bench with the engine step trace (stderr), then
# the current tree's headline kernel trace
set -o pipefail
mkdir -p gpurun_out
K8SLLM_TRACE=1 timeout -k 10 300 python bench.py --steps 4 --warmup 1 --out gpurun_out/bench_trace.json \
  > gpurun_out/bench_trace.log 2>&1 || { tail -20 gpurun_out/bench_trace.log; exit 1; }
grep "\[trace\] \(boundary\|  last\|decode\)" gpurun_out/bench_trace.log | tail -14
cut -c1-200 gpurun_out/bench_trace.json
bash scripts/gpu/run.sh prof cur > gpurun_out/prof_cur_out.txt 2>&1 || { tail -20 gpurun_out/prof_cur_out.txt; exit 1; }
head -4 gpurun_out/prof_cur_steps.txt
