# PMC counters of the decode LM-head GEMM at M = 1 and 64: row-major skinny kernel vs hipBLASLt
# (why the skinny kernel's weight bandwidth falls from 6.0 to 4.7 TB/s as M grows)
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_INSTS_MFMA GRBM_GUI_ACTIVE"
P2="TA_TA_BUSY_sum TA_DATA_STALLED_BY_TC_CYCLES_sum TD_TD_BUSY_sum TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE"
P3="TCP_PENDING_STALL_CYCLES_sum TCP_TCC_READ_REQ_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_TCR_TCP_STALL_CYCLES_sum GRBM_GUI_ACTIVE"
: > gpurun_out/lm_pmc.jsonl
for i in 1 2 3; do
  eval P=\$P$i
  timeout -s KILL 90 rocprofv3 --output-format csv --pmc $P -d gpurun_out/lpmc$i -o run -- python3 tools/bench_lm_head.py --ms 1,64 --rounds 1 --iters 32 > gpurun_out/lpmc$i.log 2>&1 || { tail -20 gpurun_out/lpmc$i.log; exit 1; }
  python3 tools/pmc_summary.py gpurun_out/lpmc$i --kernel "" | grep -v "silu\|Fill\|distribution\|copy\|rmsnorm\|add_norm\|elementwise" >> gpurun_out/lm_pmc.jsonl
done
rm -rf gpurun_out/lpmc1 gpurun_out/lpmc2 gpurun_out/lpmc3
cut -c1-900 gpurun_out/lm_pmc.jsonl
