# host side of the wave boundary on the late tree (timed waves run inside the load generator; lean
# answer path): the headline with the engine step trace, twice
set -o pipefail
mkdir -p gpurun_out
for i in ${RUNS:-1 2}; do
  K8SLLM_TRACE=1 timeout -k 10 300 python bench.py --steps 5 --warmup 2 --out gpurun_out/bench_trace2_$i.json \
    > gpurun_out/bench_trace2_$i.log 2>&1 || { tail -20 gpurun_out/bench_trace2_$i.log; exit 1; }
  grep "\[trace\] \(boundary\|  last\|prefill launch\|  k-th\)" gpurun_out/bench_trace2_$i.log | tail -13
  cut -c1-160 gpurun_out/bench_trace2_$i.json
done
