# GPU suite (engine + skinny) and the headline bench
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gputests_g.log 2>&1 || { tail -40 gpurun_out/gputests_g.log; exit 1; }
tail -2 gpurun_out/gputests_g.log
timeout -k 10 300 python bench.py --steps 5 --warmup 2 > gpurun_out/bench_g.log 2>&1 || { tail -20 gpurun_out/bench_g.log; exit 1; }
tail -1 gpurun_out/bench_g.log
