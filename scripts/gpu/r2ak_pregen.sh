# headline with the client payloads generated before the timed region (3 runs) + idle-gap analysis
set -o pipefail
mkdir -p gpurun_out
for r in 1 2 3; do
  timeout -k 10 300 python bench.py --steps 5 --warmup 2 > gpurun_out/pregen_$r.log 2>&1 || { tail -20 gpurun_out/pregen_$r.log; exit 1; }
  echo "run $r $(tail -1 gpurun_out/pregen_$r.log | cut -c70-160)"
done
bash scripts/gpu/r2aj_gaps.sh
