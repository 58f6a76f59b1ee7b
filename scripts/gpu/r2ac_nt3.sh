# 48-column tiles for the qkv slab GEMM (fills 256 CUs): numerics, microbench, headline A/B
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_skinny_rm_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/nt3_tests.log 2>&1 || { tail -30 gpurun_out/nt3_tests.log; exit 1; }
tail -1 gpurun_out/nt3_tests.log
K8SLLM_SKINNY_TILE_COLS=64 timeout -k 10 200 python tools/bench_skinny_rm.py --ms 1,64 --impls rowmajor --ops qkv --rounds 3 > gpurun_out/nt3.jsonl 2>gpurun_out/nt3.err || { tail gpurun_out/nt3.err; exit 1; }
timeout -k 10 200 python tools/bench_skinny_rm.py --ms 1,64 --impls rowmajor --ops qkv --rounds 3 >> gpurun_out/nt3.jsonl 2>>gpurun_out/nt3.err || { tail gpurun_out/nt3.err; exit 1; }
cat gpurun_out/nt3.jsonl
for r in 1 2; do
  for nt in 0 64; do
    K8SLLM_SKINNY_TILE_COLS=$nt timeout -k 10 200 python bench.py --steps 3 --warmup 1 > gpurun_out/nt3_b$nt.log 2>&1 || { tail gpurun_out/nt3_b$nt.log; exit 1; }
    echo "NT=$nt(0=auto) $(tail -1 gpurun_out/nt3_b$nt.log | cut -c70-115)"
  done
done
