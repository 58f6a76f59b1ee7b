# engine-level GPU checks of the decode GEMM integration + a headline bench
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_engine.py tests/test_real_shape_gpu.py tests/test_gemm_decode_gpu.py tests/test_tp_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/t_eng.log 2>&1; rc=$?; tail -5 gpurun_out/t_eng.log
[ $rc -eq 0 ] || { grep -E "Error|assert|FAIL" gpurun_out/t_eng.log | head -20; exit $rc; }
timeout -k 10 400 python bench.py --steps 5 --warmup 2 --out gpurun_out/bench_dec.json > gpurun_out/bench_dec.log 2>&1 || { tail -20 gpurun_out/bench_dec.log; exit 1; }
cut -c1-300 gpurun_out/bench_dec.json
K8SLLM_DECODE_GEMM=rm timeout -k 10 400 python bench.py --steps 5 --warmup 2 --out gpurun_out/bench_rm.json > gpurun_out/bench_rm.log 2>&1 || { tail -20 gpurun_out/bench_rm.log; exit 1; }
cut -c1-300 gpurun_out/bench_rm.json
