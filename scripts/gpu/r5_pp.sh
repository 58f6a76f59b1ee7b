# round 5: 8-wave ping-pong prefill GEMM - bitwise vs the 4-wave kernel, fp32 tile tests, microbench, PMC
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gemm_pp_gpu.py tests/test_gemm_tile_gpu.py -x -v --timeout 200 \
  --timeout-method thread > gpurun_out/r5_pp_tests.log 2>&1 || { tail -40 gpurun_out/r5_pp_tests.log; exit 1; }
tail -3 gpurun_out/r5_pp_tests.log
timeout -k 10 400 python tools/bench_gemm_tile.py --only qkv,o,down,gate_up+swiglu --impl w4s,pp,pp0,hipblaslt > gpurun_out/gemm_pp.jsonl 2> gpurun_out/gemm_pp.err || { tail -20 gpurun_out/gemm_pp.err; exit 1; }
cat gpurun_out/gemm_pp.jsonl | cut -c1-160
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for impl in w4s pp pp0; do
  timeout -k 10 200 python3 tools/gpu_pmc.py --pass "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_MFMA GRBM_GUI_ACTIVE" \
    --kernel gemm --out gpurun_out/pmc_pp_$impl.jsonl -- python3 tools/bench_gemm_tile.py --only gate_up+swiglu --impl $impl --rounds 1 --iters 4 \
    > gpurun_out/pmc_pp_$impl.log 2>&1 || { tail -20 gpurun_out/pmc_pp_$impl.log; exit 1; }
  cat gpurun_out/pmc_pp_$impl.jsonl
done
