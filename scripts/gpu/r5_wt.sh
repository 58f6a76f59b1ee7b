# write-through decode GEMM epilogue: parity tests, then the in-engine decode-step A/B
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gemm_decode_gpu.py tests/test_real_shape_gpu.py tests/test_decode_layout.py \
  -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/t_wt.log 2>&1 || { tail -30 gpurun_out/t_wt.log; exit 1; }
tail -1 gpurun_out/t_wt.log
timeout -k 10 600 python tools/bench_decode_step.py --switch dec_wt --rounds 3 > gpurun_out/dec_wt.jsonl 2> gpurun_out/dec_wt.err \
  || { tail -20 gpurun_out/dec_wt.err; exit 1; }
cat gpurun_out/dec_wt.jsonl
