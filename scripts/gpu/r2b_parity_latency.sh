# round 2: real-shape parity, batch-1 latency, production-timeout runs at max_tokens 2000, step bus
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_real_shape_gpu.py -x -v --timeout 300 --timeout-method thread > gpurun_out/parity.log 2>&1 || { tail -30 gpurun_out/parity.log; exit 1; }
tail -3 gpurun_out/parity.log
b() { out=$1; shift; timeout -k 10 300 python bench.py "$@" > gpurun_out/$out.log 2>&1 || { tail -20 gpurun_out/$out.log; exit 1; }; tail -1 gpurun_out/$out.log; }
b lat256 --mode latency --steps 5 --warmup 1 --max-new-tokens 256
b lat2000 --mode latency --steps 2 --warmup 1 --max-new-tokens 2000 --production
b prod2000_b64 --steps 1 --warmup 1 --max-new-tokens 2000 --production
b prod2000_b32 --steps 1 --warmup 1 --max-new-tokens 2000 --production --batch 32
timeout -k 10 120 python tools/bench_step_bus.py --steps 1500 > gpurun_out/step_bus.log 2>&1 || exit 1
grep bus gpurun_out/step_bus.log
