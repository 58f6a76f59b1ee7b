# round 6 validation, part 2: every other BASELINE config on the committed tree (podcomm, batch-1
# latency, 2000-token product defaults, Poisson 16/s, Mixtral + its trace) and a headline trace
set -o pipefail
mkdir -p gpurun_out
bash scripts/gpu/r5_configs.sh b || exit 1
bash scripts/gpu/r5_configs.sh a || exit 1
bash scripts/gpu/run.sh prof final > gpurun_out/prof_final_out.txt 2>&1 || { tail -20 gpurun_out/prof_final_out.txt; exit 1; }
head -3 gpurun_out/prof_final_steps.txt
