# batch-1 latency with and without the row-complete o projection (interleaved): at one row the
# row-complete form's activation re-read is 8 KB per workgroup, not 640 KB
set -o pipefail
mkdir -p gpurun_out
for i in 1 2; do
  for f in none rc; do
    timeout -k 10 300 python bench.py --mode latency --steps 5 --warmup 1 --decode-fusion $f \
      --out gpurun_out/latrc_${f}_$i.json > gpurun_out/latrc_${f}_$i.log 2>&1 || { tail -20 gpurun_out/latrc_${f}_$i.log; exit 1; }
  done
  python3 -c "import json;f=lambda n:json.load(open(n));a=f('gpurun_out/latrc_rc_$i.json');b=f('gpurun_out/latrc_none_$i.json');print('rc', a['p50_latency_ms'], a['tpot_ms'], 'none', b['p50_latency_ms'], b['tpot_ms'])"
done
