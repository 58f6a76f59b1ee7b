# round 6: is the tile GEMM's per-tile gap to hipBLASLt the XOR-permuted DMA source addresses (TA)?
# K8SLLM_TILE_NOXOR=1 makes the DMA read each row's 16-B chunks in order (numerically wrong: the LDS
# reads stay XOR-addressed, so the LDS access pattern is unchanged) - timing only
set -o pipefail
mkdir -p gpurun_out
for shp in "4096 4096" "28672 4096" "4096 14336"; do
  set -- $shp
  bash scripts/gpu/run.sh tool xor_$1_$2 tools/gemm_k_sweep.py --n $1 --ks $2 --packed --rounds 3 || exit 1
  K8SLLM_TILE_NOXOR=1 bash scripts/gpu/run.sh tool noxor_$1_$2 tools/gemm_k_sweep.py --n $1 --ks $2 --packed --rounds 3 || exit 1
done
