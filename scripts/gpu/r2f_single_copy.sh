# single resident weight copy (row-major skinny decode): full GPU suite + headline bench
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/gputests_f.log 2>&1 || { tail -40 gpurun_out/gputests_f.log; exit 1; }
tail -3 gpurun_out/gputests_f.log
timeout -k 10 300 python bench.py --steps 5 --warmup 2 > gpurun_out/bench_f.log 2>&1 || { tail -20 gpurun_out/bench_f.log; exit 1; }
tail -1 gpurun_out/bench_f.log
K8SLLM_SKINNY_LAYOUT=packed timeout -k 10 300 python bench.py --steps 5 --warmup 2 > gpurun_out/bench_f_packed.log 2>&1 || { tail -20 gpurun_out/bench_f_packed.log; exit 1; }
tail -1 gpurun_out/bench_f_packed.log
