# round 6: ONE weight layout - the full GPU suite (packed / SWIGLU8 tile tests,
# one-layout parity), smoke, the headline with one layout vs two (A/B/A), a kernel trace
set -o pipefail
mkdir -p gpurun_out
bash scripts/gpu/run.sh suite || exit 1
bash scripts/gpu/run.sh bench two1 --steps 5 --warmup 2 --layout two || exit 1
bash scripts/gpu/run.sh bench one2 --steps 5 --warmup 2 --layout one || exit 1
bash scripts/gpu/run.sh prof one > gpurun_out/prof_one_out.txt 2>&1 || { tail -20 gpurun_out/prof_one_out.txt; exit 1; }
head -12 gpurun_out/prof_one_steps.txt
