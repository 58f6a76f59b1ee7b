# flash prefill: staggered halves vs lockstep, interleaved processes; then the flash GPU tests
set -o pipefail
mkdir -p gpurun_out
rm -f gpurun_out/flash_ab.jsonl
timeout -k 10 300 python -u -m pytest tests/test_ops_gpu.py tests/test_real_shape_gpu.py tests/test_engine.py -m gpu -x -q --timeout 200 --timeout-method thread -k "flash or prefill or chunked or real_shape" > gpurun_out/t_flash.log 2>&1 || { tail -30 gpurun_out/t_flash.log; exit 1; }
tail -2 gpurun_out/t_flash.log
for r in 1 2; do
  for st in 0 1; do
    for sl in 10:1609 4:4000 2:8192; do
      K8SLLM_FLASH_STAGGER=$st timeout -k 10 120 python tools/bench_prefill_attn.py --seqs ${sl%%:*} --len ${sl##*:} 2>> gpurun_out/flash_ab.err | grep paged | sed "s/^{/{\"stagger\": $st, /" >> gpurun_out/flash_ab.jsonl || { tail -5 gpurun_out/flash_ab.err; exit 1; }
    done
  done
done
cat gpurun_out/flash_ab.jsonl
