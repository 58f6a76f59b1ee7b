# kernel traces of the late tree: the headline (64 rows) and batch-1 latency (row-complete o,
# in-launch attention merge: no paged_decode_reduce kernel)
set -o pipefail
mkdir -p gpurun_out
bash scripts/gpu/run.sh prof late > gpurun_out/prof_late_out.txt 2>&1 || { tail -20 gpurun_out/prof_late_out.txt; exit 1; }
head -3 gpurun_out/prof_late_steps.txt
bash scripts/gpu/run.sh prof latlate --mode latency --steps 3 --warmup 1 > gpurun_out/prof_latlate_out.txt 2>&1 \
  || { tail -20 gpurun_out/prof_latlate_out.txt; exit 1; }
head -3 gpurun_out/prof_latlate_steps.txt
grep -c "paged_decode_reduce" gpurun_out/prof_latlate_summary.md || true
