set -o pipefail
mkdir -p gpurun_out
run() { timeout -k 10 300 python bench.py "$@"; }
run --steps 4 --warmup 1 --mixed-prefill-tokens 16384 > gpurun_out/b_mixed16k.log 2>&1 || exit 1
tail -1 gpurun_out/b_mixed16k.log
run --steps 4 --warmup 1 --mixed-prefill-tokens 0 > gpurun_out/b_mixed0.log 2>&1 || exit 1
tail -1 gpurun_out/b_mixed0.log
run --steps 2 --warmup 1 --mode poisson --rate 12 --batch 64 --mixed-prefill-tokens 16384 > gpurun_out/b_pois16k.log 2>&1 || exit 1
tail -1 gpurun_out/b_pois16k.log
run --steps 2 --warmup 1 --mode poisson --rate 12 --batch 64 --mixed-prefill-tokens 2048 > gpurun_out/b_pois2k.log 2>&1 || exit 1
tail -1 gpurun_out/b_pois2k.log
run --steps 2 --warmup 1 --mode poisson --rate 12 --batch 64 --mixed-prefill-tokens 0 > gpurun_out/b_pois0.log 2>&1 || exit 1
tail -1 gpurun_out/b_pois0.log
