# PMC counters: tile GEMM vs hipBLASLt on the gate_up prefill shape (one pass per counter group)
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE"
P2="SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_INSTS_MFMA SQ_INSTS_SALU SQ_INSTS_VALU SQ_INSTS_VALU_TRANS_F32 SQ_LDS_IDX_ACTIVE"
for i in 1 2; do
  eval P=\$P$i
  timeout -s KILL 120 rocprofv3 --output-format csv --pmc $P -d gpurun_out/gpmc$i -o run -- python3 tools/bench_gemm_tile.py --only o,gate_up+swiglu --impl tile,hipblaslt_gemm_only,hipblaslt --rounds 1 --iters 4 > gpurun_out/gpmc$i.log 2>&1 || { tail -20 gpurun_out/gpmc$i.log; exit 1; }
  python3 tools/pmc_summary.py gpurun_out/gpmc$i --kernel "" >> gpurun_out/gemm_pmc.jsonl
done
rm -rf gpurun_out/gpmc1 gpurun_out/gpmc2
grep -v "silu\|Fill\|distribution\|copy" gpurun_out/gemm_pmc.jsonl | cut -c1-1200
