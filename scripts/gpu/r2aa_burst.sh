# burst-aware mixing (prefill-first while the backlog exceeds a step, <= 8 stalled steps) vs
# always-mix (K8SLLM_DECODE_STALL_STEPS=0): headline wave and poisson 12 q/s, interleaved
set -o pipefail
mkdir -p gpurun_out
run() { timeout -k 10 300 python bench.py "$@"; }
for r in 1 2; do
  for st in 8 0; do
    K8SLLM_DECODE_STALL_STEPS=$st run --steps 3 --warmup 1 > gpurun_out/burst_w_$st.log 2>&1 || { tail gpurun_out/burst_w_$st.log; exit 1; }
    echo "wave stall=$st $(tail -1 gpurun_out/burst_w_$st.log | cut -c70-120)"
    cp gpurun_out/burst_w_$st.log gpurun_out/burst_w_${st}_r$r.log
  done
done
for st in 8 0; do
  K8SLLM_DECODE_STALL_STEPS=$st run --steps 2 --warmup 1 --mode poisson --rate 12 --batch 64 > gpurun_out/burst_p_$st.log 2>&1 || { tail gpurun_out/burst_p_$st.log; exit 1; }
  tail -1 gpurun_out/burst_p_$st.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('poisson stall=$st', {k: d.get(k) for k in ('value','p50_latency_ms','p99_latency_ms','ttft_p50_ms','tpot_p50_ms','tpot_p99_ms')})"
done
