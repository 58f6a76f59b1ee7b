# decode seam fusion with the weight ring filled before the norm phase: kernel trace + interleaved
# headline A/B (default vs --decode-fusion seam)
set -o pipefail
mkdir -p gpurun_out
bash scripts/gpu/run.sh prof seam2 --decode-fusion seam > gpurun_out/prof_seam2_out.txt 2>&1 \
  || { tail -20 gpurun_out/prof_seam2_out.txt; exit 1; }
head -2 gpurun_out/prof_seam2_steps.txt
for i in 1 2; do
  for f in none seam; do
    timeout -k 10 300 python bench.py --steps 4 --warmup 1 --decode-fusion $f --out gpurun_out/bench_seam2_${f}_$i.json \
      > gpurun_out/bench_seam2_${f}_$i.log 2>&1 || { tail -20 gpurun_out/bench_seam2_${f}_$i.log; exit 1; }
  done
  python3 -c "import json;print('seam', json.load(open('gpurun_out/bench_seam2_seam_$i.json'))['value'], 'none', json.load(open('gpurun_out/bench_seam2_none_$i.json'))['value'])"
done
