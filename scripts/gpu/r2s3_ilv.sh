# skinny row-major GEMM with the refill DMA pieces interleaved among the MFMAs vs without
# (K8SLLM_SKINNY_ILV=0), same box, alternating processes: parity + timing
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest tests/test_skinny_rm_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/ilv_tests.log 2>&1 || { tail -30 gpurun_out/ilv_tests.log; exit 1; }
tail -1 gpurun_out/ilv_tests.log
: > gpurun_out/ilv_ab.jsonl
for r in 1 2; do
  for v in 1 0; do
    K8SLLM_SKINNY_ILV=$v timeout -k 10 200 python -u tools/bench_skinny_rm.py --ops qkv,o,gate_up,down --ms 1,64 --impls rowmajor --rounds 2 2>/dev/null | sed "s/^{/{\"ilv\": $v, \"round\": $r, /" >> gpurun_out/ilv_ab.jsonl || exit 1
  done
done
cat gpurun_out/ilv_ab.jsonl
