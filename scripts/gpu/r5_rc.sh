# round 5: row-complete o projection - numerics, microbench, headline A/B, trace
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gemm_decode_gpu.py tests/test_real_shape_gpu.py -x -v --timeout 200 \
  --timeout-method thread > gpurun_out/r5_rc_tests.log 2>&1 || { tail -40 gpurun_out/r5_rc_tests.log; exit 1; }
tail -3 gpurun_out/r5_rc_tests.log
timeout -k 10 300 python tools/bench_dec_rc.py > gpurun_out/dec_rc.jsonl 2> gpurun_out/dec_rc.err || { tail -20 gpurun_out/dec_rc.err; exit 1; }
cat gpurun_out/dec_rc.jsonl | cut -c1-80
for i in 1 2; do
  K8SLLM_DEC_RC=1 timeout -k 10 300 python bench.py --steps 4 --warmup 1 --out gpurun_out/bench_rc_on_$i.json \
    > gpurun_out/bench_rc_on_$i.log 2>&1 || { tail -20 gpurun_out/bench_rc_on_$i.log; exit 1; }
  K8SLLM_DEC_RC=0 timeout -k 10 300 python bench.py --steps 4 --warmup 1 --out gpurun_out/bench_rc_off_$i.json \
    > gpurun_out/bench_rc_off_$i.log 2>&1 || { tail -20 gpurun_out/bench_rc_off_$i.log; exit 1; }
  python3 -c "import json;a=json.load(open('gpurun_out/bench_rc_on_$i.json'));b=json.load(open('gpurun_out/bench_rc_off_$i.json'));print('rc',a['value'],'slabs',b['value'])"
done
bash scripts/gpu/run.sh prof rc > gpurun_out/prof_rc_out.txt 2>&1 || { tail -20 gpurun_out/prof_rc_out.txt; exit 1; }
head -3 gpurun_out/prof_rc_steps.txt
