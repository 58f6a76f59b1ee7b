# rm skinny GEMM with the A operand straight to VGPRs: numerics, microbench A/B, headline A/B
set -o pipefail
mkdir -p gpurun_out
K8SLLM_SKINNY_AREG=1 timeout -k 10 300 python -u -m pytest tests/test_skinny_rm_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/areg_tests.log 2>&1 || { tail -30 gpurun_out/areg_tests.log; exit 1; }
tail -1 gpurun_out/areg_tests.log
: > gpurun_out/areg.jsonl
for a in 0 1; do
  K8SLLM_SKINNY_AREG=$a timeout -k 10 300 python tools/bench_skinny_rm.py --ms 1,64 --impls rowmajor --rounds 2 > gpurun_out/areg_$a.jsonl 2>gpurun_out/areg.err || { tail gpurun_out/areg.err; exit 1; }
  echo "AREG=$a"; cat gpurun_out/areg_$a.jsonl
done
for r in 1 2; do
  for a in 1 0; do
    K8SLLM_SKINNY_AREG=$a timeout -k 10 200 python bench.py --steps 3 --warmup 1 > gpurun_out/areg_b$a.log 2>&1 || { tail gpurun_out/areg_b$a.log; exit 1; }
    echo "headline AREG=$a $(tail -1 gpurun_out/areg_b$a.log | cut -c70-115)"
    cp gpurun_out/areg_b$a.log gpurun_out/areg_b${a}_r$r.log
  done
done
