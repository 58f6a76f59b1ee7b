# PMC counters of the paged prefill kernels (v1 vs v2), one pass per counter group
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE"
P2="SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_INSTS_MFMA SQ_INSTS_SALU SQ_INSTS_VALU SQ_INSTS_VALU_TRANS_F32 SQ_LDS_IDX_ACTIVE"
for v in v1 v2; do
  timeout -s KILL 90 rocprofv3 --output-format csv --pmc $P1 -d gpurun_out/pmc1_$v -o run -- python3 tools/bench_prefill_attn.py --only $v --iters 5 > gpurun_out/pmc1_$v.log 2>&1 || { tail -20 gpurun_out/pmc1_$v.log; exit 1; }
  timeout -s KILL 90 rocprofv3 --output-format csv --pmc $P2 -d gpurun_out/pmc2_$v -o run -- python3 tools/bench_prefill_attn.py --only $v --iters 5 > gpurun_out/pmc2_$v.log 2>&1 || { tail -20 gpurun_out/pmc2_$v.log; exit 1; }
  python3 tools/pmc_summary.py gpurun_out/pmc1_$v --kernel flash_prefill > gpurun_out/pmc_$v.jsonl
  python3 tools/pmc_summary.py gpurun_out/pmc2_$v --kernel flash_prefill >> gpurun_out/pmc_$v.jsonl
  cat gpurun_out/pmc_$v.jsonl
done
find gpurun_out/pmc1_v2 | head; rm -rf gpurun_out/pmc1_* gpurun_out/pmc2_*
timeout -k 10 200 python tools/bench_prefill_attn.py > gpurun_out/pf2_bench.jsonl 2>gpurun_out/pf2_bench.err || exit 1
cat gpurun_out/pf2_bench.jsonl
