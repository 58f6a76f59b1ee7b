# in-launch split merge for paged decode: numerics, batch-1 latency A/B, headline check
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_ops_gpu.py -k "decode" -x -q --timeout 120 --timeout-method thread > gpurun_out/merge_tests.log 2>&1 || { tail -30 gpurun_out/merge_tests.log; exit 1; }
tail -1 gpurun_out/merge_tests.log
for r in 1 2; do
  for m in 1 0; do
    K8SLLM_DECODE_MERGE=$m timeout -k 10 200 python bench.py --mode latency --batch 1 --steps 6 --warmup 2 > gpurun_out/merge_lat$m.log 2>&1 || { tail gpurun_out/merge_lat$m.log; exit 1; }
    echo "merge=$m $(tail -1 gpurun_out/merge_lat$m.log | cut -c70-140)"
    cp gpurun_out/merge_lat$m.log gpurun_out/merge_lat${m}_r$r.log
  done
done
timeout -k 10 200 python bench.py --steps 3 --warmup 1 > gpurun_out/merge_head.log 2>&1 || { tail gpurun_out/merge_head.log; exit 1; }
echo "headline $(tail -1 gpurun_out/merge_head.log | cut -c70-140)"
