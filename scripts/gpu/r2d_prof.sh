# kernel trace of the headline bench (2 timed waves) + paged decode / prefill attention microbenches
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r2d -o run -- python3 bench.py --steps 2 --warmup 1 > gpurun_out/prof_r2d.log 2>&1 || { tail -30 gpurun_out/prof_r2d.log; exit 1; }
tail -1 gpurun_out/prof_r2d.log
f=$(find gpurun_out/prof_r2d -name "*results.db" | head -1)
python3 tools/rocpd_summary.py $f --top 40 --title "r2d headline bench" > gpurun_out/prof_r2d_summary.md
timeout -k 10 200 python3 tools/bench_prefill_attn.py > gpurun_out/prefill_attn.log 2>&1 || { tail -30 gpurun_out/prefill_attn.log; exit 1; }
cat gpurun_out/prefill_attn.log | tail -15
