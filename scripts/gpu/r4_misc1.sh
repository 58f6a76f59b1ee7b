# wave-boundary trace, all-tile vs default routing headline A/B (3 interleaved pairs), flash prefill
# 4 x 8000 / 10 x 1609 timings and an MFMA-busy PMC pass over flash v2
set -o pipefail
mkdir -p gpurun_out
K8SLLM_TRACE=1 timeout -k 10 300 python bench.py --steps 3 --warmup 1 --out gpurun_out/bench_trace.json > gpurun_out/bench_trace.log 2>&1 || { tail -20 gpurun_out/bench_trace.log; exit 1; }
grep "\[trace\]" gpurun_out/bench_trace.log | grep -v "prefill +" || true
for r in 1 2 3; do
  for mode in auto tile; do
    K8SLLM_PREFILL_GEMM=$mode timeout -k 10 300 python bench.py --steps 4 --warmup 2 --out gpurun_out/bench_pg2_${mode}_$r.json > gpurun_out/bench_pg2_${mode}_$r.log 2>&1 || { tail -20 gpurun_out/bench_pg2_${mode}_$r.log; exit 1; }
    echo "$mode $r $(cut -c80-110 gpurun_out/bench_pg2_${mode}_$r.json)"
  done
done
timeout -k 10 120 python tools/bench_prefill_attn.py --seqs 4 --len 8000 > gpurun_out/flash_4x8000.jsonl 2>&1 || { tail -20 gpurun_out/flash_4x8000.jsonl; exit 1; }
timeout -k 10 120 python tools/bench_prefill_attn.py --seqs 10 --len 1609 >> gpurun_out/flash_4x8000.jsonl 2>&1 || { tail -20 gpurun_out/flash_4x8000.jsonl; exit 1; }
cat gpurun_out/flash_4x8000.jsonl
root=$PWD
cd /tmp && export TMPDIR=/tmp && cd "$root"
timeout -k 10 200 python3 tools/gpu_pmc.py --pass "GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_MFMA SQ_INSTS_VALU" --kernel flash_prefill --out gpurun_out/pmc_flash_8k.jsonl -- python3 tools/bench_prefill_attn.py --seqs 4 --len 8000 --iters 5 || { echo "pmc failed"; exit 1; }
cat gpurun_out/pmc_flash_8k.jsonl
timeout -k 10 200 python3 tools/gpu_pmc.py --pass "GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_MFMA SQ_INSTS_VALU" --kernel flash_prefill --out gpurun_out/pmc_flash_1609.jsonl -- python3 tools/bench_prefill_attn.py --seqs 10 --len 1609 --iters 5 || { echo "pmc failed"; exit 1; }
cat gpurun_out/pmc_flash_1609.jsonl
timeout -k 10 400 python bench.py --production --max-new-tokens 2000 --steps 2 --warmup 1 --out gpurun_out/prod2000_kv.json > gpurun_out/prod2000_kv.log 2>&1 || { tail -20 gpurun_out/prod2000_kv.log; exit 1; }
cut -c1-1500 gpurun_out/prod2000_kv.json
