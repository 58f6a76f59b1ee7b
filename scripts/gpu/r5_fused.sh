# round 5: fused add-RMSNorm decode GEMMs - numerics, then headline A/B (fused vs two launches) and a trace
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gemm_decode_gpu.py tests/test_real_shape_gpu.py -x -v --timeout 200 \
  --timeout-method thread > gpurun_out/r5_fused_tests.log 2>&1 || { tail -40 gpurun_out/r5_fused_tests.log; exit 1; }
tail -3 gpurun_out/r5_fused_tests.log
for i in 1 2; do
  K8SLLM_FUSED_NORM=1 timeout -k 10 300 python bench.py --steps 4 --warmup 1 --out gpurun_out/bench_fn_on_$i.json \
    > gpurun_out/bench_fn_on_$i.log 2>&1 || { tail -20 gpurun_out/bench_fn_on_$i.log; exit 1; }
  K8SLLM_FUSED_NORM=0 timeout -k 10 300 python bench.py --steps 4 --warmup 1 --out gpurun_out/bench_fn_off_$i.json \
    > gpurun_out/bench_fn_off_$i.log 2>&1 || { tail -20 gpurun_out/bench_fn_off_$i.log; exit 1; }
  python3 -c "import json;a=json.load(open('gpurun_out/bench_fn_on_$i.json'));b=json.load(open('gpurun_out/bench_fn_off_$i.json'));print('fused',a['value'],'unfused',b['value'])"
done
bash scripts/gpu/run.sh prof fn > gpurun_out/prof_fn_out.txt 2>&1 || { tail -20 gpurun_out/prof_fn_out.txt; exit 1; }
head -3 gpurun_out/prof_fn_steps.txt
