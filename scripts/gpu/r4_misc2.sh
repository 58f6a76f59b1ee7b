# product-default serving with the context-aware admission model, the headline with the all-tile
# routing default, and its kernel trace
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python bench.py --production --max-new-tokens 2000 --steps 2 --warmup 1 --out gpurun_out/prod2000_kv2.json > gpurun_out/prod2000_kv2.log 2>&1 || { tail -20 gpurun_out/prod2000_kv2.log; exit 1; }
cut -c1-300 gpurun_out/prod2000_kv2.json; python3 -c "import json;d=json.load(open('gpurun_out/prod2000_kv2.json'));print(d['requests'], d['tpot_model_ms'].get('kv_fit'), d['ttft_ms'], d['tpot_ms'], d['p99_latency_ms'])"
timeout -k 10 300 python bench.py --steps 5 --warmup 2 --out gpurun_out/bench_tile_default.json > gpurun_out/bench_tile_default.log 2>&1 || { tail -20 gpurun_out/bench_tile_default.log; exit 1; }
cut -c1-200 gpurun_out/bench_tile_default.json
bash scripts/gpu/run.sh prof tile1 > gpurun_out/prof_tile1_out.txt 2>&1 || { tail -20 gpurun_out/prof_tile1_out.txt; exit 1; }
head -3 gpurun_out/prof_tile1_steps.txt; head -16 gpurun_out/prof_tile1_summary.md
