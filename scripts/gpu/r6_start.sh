# round 6 start: GPU suite + smoke + headline on the inherited tree, then where the prefill tile
# GEMM loses to hipBLASLt: a K sweep (fixed vs per-k cost) and PMC passes over both at the o shape
set -o pipefail
mkdir -p gpurun_out
bash scripts/gpu/run.sh suite || exit 1
bash scripts/gpu/run.sh tool ksweep tools/gemm_k_sweep.py --n 4096 || exit 1
bash scripts/gpu/run.sh tool ksweep14k tools/gemm_k_sweep.py --n 14336 --ks 1024,2048,4096 --rounds 2 || exit 1
bash scripts/gpu/run.sh pmc gemm_o "" \
  "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_ANY SQ_INSTS_MFMA GRBM_GUI_ACTIVE" \
  "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_LDS_ADDR_CONFLICT SQ_LDS_DATA_FIFO_FULL SQ_LDS_CMD_FIFO_FULL SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_LDS_UNALIGNED_STALL GRBM_GUI_ACTIVE" \
  "TCC_HIT_sum TCC_MISS_sum TA_TA_BUSY_sum SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_INSTS_VALU GRBM_GUI_ACTIVE" \
  -- python3 tools/bench_gemm_tile.py --only o --impl w4s,hipblaslt --rounds 1 --iters 8 || exit 1
