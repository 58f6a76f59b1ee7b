# the seam GEMM with its weight ring issued before the seam wait (waves 1..3 before the spin,
# wave 0 after it): bit-identity against the two-launch path, then decode-step A/B at 64 and 1 rows
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_gemm_decode_gpu.py -k "fused_norm or rc_matches" > gpurun_out/se_tests.log 2>&1
echo "tests rc=$?"; tail -2 gpurun_out/se_tests.log
grep -q " passed" gpurun_out/se_tests.log && ! grep -q "failed" gpurun_out/se_tests.log || exit 1
timeout -k 10 400 python -u tools/bench_decode_step.py --switch seam_auto_rc --rows 64,1 --rounds 3 --tokens 64 \
  > gpurun_out/se_ab.jsonl 2> gpurun_out/se_ab.err || { tail -20 gpurun_out/se_ab.err; exit 1; }
grep on_median gpurun_out/se_ab.jsonl
