# end-of-round evidence: full GPU suite + smoke + headline, a second headline, the kernel trace,
# and the product-default serving record
set -o pipefail
mkdir -p gpurun_out
bash scripts/gpu/run.sh suite || exit 1
timeout -k 10 300 python bench.py --steps 5 --warmup 2 --out gpurun_out/bench_final2.json > gpurun_out/bench_final2.log 2>&1 || { tail -20 gpurun_out/bench_final2.log; exit 1; }
cut -c1-200 gpurun_out/bench_final2.json
bash scripts/gpu/run.sh prof final > gpurun_out/prof_final_out.txt 2>&1 || { tail -20 gpurun_out/prof_final_out.txt; exit 1; }
head -2 gpurun_out/prof_final_steps.txt
timeout -k 10 400 python bench.py --production --max-new-tokens 2000 --steps 2 --warmup 1 --out gpurun_out/prod_final.json > gpurun_out/prod_final.log 2>&1 || { tail -20 gpurun_out/prod_final.log; exit 1; }
python3 -c "import json;d=json.load(open('gpurun_out/prod_final.json'));print(d['value'], d['requests'], d['p99_latency_ms'])"
