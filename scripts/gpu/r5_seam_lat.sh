# batch-1 latency with and without the seam fusion (interleaved)
set -o pipefail
mkdir -p gpurun_out
for i in 1 2; do
  for f in none seam; do
    timeout -k 10 300 python bench.py --mode latency --steps 5 --warmup 1 --decode-fusion $f \
      --out gpurun_out/lat_${f}_$i.json > gpurun_out/lat_${f}_$i.log 2>&1 || { tail -20 gpurun_out/lat_${f}_$i.log; exit 1; }
  done
  python3 -c "import json;f=lambda n:json.load(open(n));a=f('gpurun_out/lat_seam_$i.json');b=f('gpurun_out/lat_none_$i.json');print('seam', a['p50_latency_ms'], a['tpot_ms'], 'none', b['p50_latency_ms'], b['tpot_ms'])"
done
