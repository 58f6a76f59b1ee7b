# round-4 serving records: batch-1 latency, the product-default 2000-token answers under the
# reference timeouts at 64 concurrent, and the W = 8 IPC collective probe on the one GPU
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_skinny_rm_gpu.py tests/test_tp_gpu.py tests/test_ops_gpu.py tests/test_real_shape_gpu.py -m gpu -x -q --timeout 240 --timeout-method thread -k "grouped or ep2 or flash or prefill" > gpurun_out/t_grp.log 2>&1 || { tail -30 gpurun_out/t_grp.log; exit 1; }
tail -2 gpurun_out/t_grp.log
for sl in 10:1609 4:4000 2:8192 1:8000; do
  timeout -k 10 120 python tools/bench_prefill_attn.py --seqs ${sl%%:*} --len ${sl##*:} >> gpurun_out/flash_r4.jsonl 2>> gpurun_out/flash_r4.err || { tail -5 gpurun_out/flash_r4.err; exit 1; }
done
cat gpurun_out/flash_r4.jsonl
timeout -k 10 300 python bench.py --mode latency --steps 5 --warmup 1 --out gpurun_out/lat256.json > gpurun_out/lat256.log 2>&1 || { tail -20 gpurun_out/lat256.log; exit 1; }
cut -c1-400 gpurun_out/lat256.json
timeout -k 10 400 python bench.py --production --max-new-tokens 2000 --steps 2 --warmup 1 --out gpurun_out/prod2000_b64.json > gpurun_out/prod2000_b64.log 2>&1 || { tail -20 gpurun_out/prod2000_b64.log; exit 1; }
cut -c1-1200 gpurun_out/prod2000_b64.json
timeout -k 10 200 python tools/probe_custom_ar_w8.py > gpurun_out/w8.json 2> gpurun_out/w8.err || { tail -5 gpurun_out/w8.err; exit 1; }
cat gpurun_out/w8.json
