# balanced decode splits (chunks per split): numerics with the mode on, then headline A/B
set -o pipefail
mkdir -p gpurun_out
K8SLLM_DECODE_CPS=2 timeout -k 10 300 python -u -m pytest tests/test_ops_gpu.py -k "decode" -x -q --timeout 120 --timeout-method thread > gpurun_out/cps_tests.log 2>&1 || { tail -30 gpurun_out/cps_tests.log; exit 1; }
tail -1 gpurun_out/cps_tests.log
: > gpurun_out/cps.jsonl
for r in 1 2; do
for c in 0 2 4 8; do
  K8SLLM_DECODE_CPS=$c timeout -k 10 200 python bench.py --steps 3 --warmup 1 > gpurun_out/cps_$c.log 2>&1 || { tail -20 gpurun_out/cps_$c.log; exit 1; }
  echo "{\"cps\": $c, \"round\": $r, \"line\": $(tail -1 gpurun_out/cps_$c.log)}" >> gpurun_out/cps.jsonl
  echo "cps=$c $(tail -1 gpurun_out/cps_$c.log | cut -c70-140)"
done
done
