# round 6: ONE weight layout - the tile GEMM's packed / SWIGLU8 tests, the
# real-shape and decode suites, smoke, then the headline with one layout vs two (A/B/A)
set -o pipefail
mkdir -p gpurun_out
bash scripts/gpu/run.sh tests 'gemm_tile or real_shape or tile_real or decode or one_layout' || exit 1
timeout -k 10 300 python -u __graft_entry__.py smoke > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 1; }
tail -2 gpurun_out/smoke.log
bash scripts/gpu/run.sh bench one1 --steps 5 --warmup 2 --layout one || exit 1
bash scripts/gpu/run.sh bench two1 --steps 5 --warmup 2 --layout two || exit 1
bash scripts/gpu/run.sh bench one2 --steps 5 --warmup 2 --layout one || exit 1
