# PMC of the paged flash prefill after the q-block order and softmax overlap changes
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for sh in "10 1609" "4 8000"; do
  set -- $sh
  PLAIN=0 timeout -k 10 200 python3 tools/gpu_pmc.py --pass "GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_MFMA SQ_INSTS_VALU" --kernel flash_prefill_paged --out gpurun_out/pmc_flash_r4b_$1x$2.jsonl -- python3 tools/bench_prefill_attn.py --seqs $1 --len $2 --iters 5 --orders seq || { echo "pmc failed"; exit 1; }
  cat gpurun_out/pmc_flash_r4b_$1x$2.jsonl
done
