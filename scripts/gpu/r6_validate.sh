# round 6 cleanup validation: GPU suite (custom-AR self-test, numeric smoke) + headline, the
# smoke's fault-injection check, and a kernel trace of the headline (idle-gap census)
set -o pipefail
mkdir -p gpurun_out
bash scripts/gpu/run.sh suite || exit 1
timeout -k 10 300 python -u tools/smoke_fault.py > gpurun_out/smoke_fault.log 2>&1 || { tail -20 gpurun_out/smoke_fault.log; exit 1; }
tail -1 gpurun_out/smoke_fault.log
bash scripts/gpu/run.sh prof r6a > gpurun_out/prof_r6a_out.txt 2>&1 || { tail -20 gpurun_out/prof_r6a_out.txt; exit 1; }
head -30 gpurun_out/prof_r6a_steps.txt
