# round-4 GPU checks: real-shape tile parity, W = 2 / 4 IPC collectives and TP engine on one GPU,
# then an in-engine A/B of the decode o / down split-K factor
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_tile_real_shapes_gpu.py tests/test_custom_ar.py -m gpu -x -v --timeout 240 --timeout-method thread > gpurun_out/t_r4a.log 2>&1; rc=$?
grep -E "PASS|FAIL|ERROR|passed|failed" gpurun_out/t_r4a.log | tail -30
[ $rc -eq 0 ] || { grep -E "Error|assert" gpurun_out/t_r4a.log | head -20; exit $rc; }
for t in s8 s4; do
  if [ $t = s4 ]; then export K8SLLM_DEC_TABLE="4096,4096,0=4,1,4,16;4096,14336,0=4,1,4,16"; fi
  timeout -k 10 400 python bench.py --steps 5 --warmup 2 --out gpurun_out/bench_$t.json > gpurun_out/bench_$t.log 2>&1 || { tail -20 gpurun_out/bench_$t.log; exit 1; }
  cut -c1-200 gpurun_out/bench_$t.json
done
