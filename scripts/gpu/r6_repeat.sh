# round 6: the headline three times on one box (run-to-run spread of the final tree)
set -o pipefail
mkdir -p gpurun_out
for r in 1 2 3; do
  bash scripts/gpu/run.sh bench rep$r --steps 5 --warmup 2 || exit 1
done
