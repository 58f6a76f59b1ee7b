# round 6: tile GEMM vs hipBLASLt over the number of tile waves (M) at N = K = 4096
set -o pipefail
mkdir -p gpurun_out
for m in 4096 16384 65536; do
  bash scripts/gpu/run.sh tool msw_$m tools/gemm_k_sweep.py --m $m --n 4096 --ks 4096 --algos 1,2 --rounds 3 || exit 1
done
