# round 6: tile GEMM over fragment-packed weights (the decode layout) vs row-major; flash prefill
# staggered (ping-pong) main loop vs unstaggered; then the cleanup validation (suite + numeric
# smoke + its fault injection + headline kernel trace)
set -o pipefail
mkdir -p gpurun_out
bash scripts/gpu/run.sh tests 'gemm_tile or prefill or flash' || exit 1
bash scripts/gpu/run.sh tool pk_o tools/gemm_k_sweep.py --n 4096 --ks 4096 --packed --rounds 3 || exit 1
bash scripts/gpu/run.sh tool pk_gu tools/gemm_k_sweep.py --n 14336 --ks 4096 --packed --rounds 2 || exit 1
bash scripts/gpu/run.sh tool pk_d tools/gemm_k_sweep.py --n 4096 --ks 14336 --packed --rounds 2 || exit 1
bash scripts/gpu/run.sh tool fl_10x1609 tools/bench_prefill_attn.py --seqs 10 --len 1609 --stag 0,1 || exit 1
bash scripts/gpu/run.sh tool fl_64x1609 tools/bench_prefill_attn.py --seqs 64 --len 1609 --stag 0,1 --iters 5 || exit 1
bash scripts/gpu/run.sh tool fl_8k tools/bench_prefill_attn.py --seqs 2 --len 8192 --stag 0,1 --iters 5 || exit 1
bash scripts/gpu/run.sh tool fl_70b tools/bench_prefill_attn.py --seqs 10 --len 1609 --hq 64 --hkv 8 --stag 0,1 || exit 1
bash scripts/gpu/run.sh tool fl_70b8k tools/bench_prefill_attn.py --seqs 2 --len 8192 --hq 64 --hkv 8 --stag 0,1 --iters 5 || exit 1
bash scripts/gpu/r6_validate.sh || exit 1
