# prefill step budget A/B on the headline: 16384 (default) vs 32768 vs 24576 tokens per step
set -o pipefail
mkdir -p gpurun_out
for i in 1 2; do
  for t in ${BUDGETS:-16384 32768 24576}; do
    timeout -k 10 300 python bench.py --steps 5 --warmup 2 --max-prefill-tokens $t --out gpurun_out/pf_${t}_$i.json \
      > gpurun_out/pf_${t}_$i.log 2>&1 || { tail -20 gpurun_out/pf_${t}_$i.log; exit 1; }
    python3 -c "import json;d=json.load(open('gpurun_out/pf_${t}_$i.json'));print('budget $t round $i', d['value'], d['p50_latency_ms'], d['prefill_steps'])"
  done
done
