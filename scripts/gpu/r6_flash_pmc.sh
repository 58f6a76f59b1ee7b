# round 6: PMC of the paged flash prefill (v2) at the VERDICT shapes: MFMA busy, VALU / MFMA mix, LDS waits
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export PLAIN=0
for sh in "10 1609 32" "2 8192 32" "10 1609 64"; do
  set -- $sh
  timeout -k 10 200 python3 tools/gpu_pmc.py --pass "GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_MFMA SQ_INSTS_VALU" --kernel flash_prefill_paged --out gpurun_out/pmc_flash_r6_$1x$2_hq$3.jsonl -- python3 tools/bench_prefill_attn.py --seqs $1 --len $2 --hq $3 --iters 5 || { echo "pmc failed"; exit 1; }
  cat gpurun_out/pmc_flash_r6_$1x$2_hq$3.jsonl
done
