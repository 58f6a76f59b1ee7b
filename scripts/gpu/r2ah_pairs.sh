# flash prefill v2, one barrier per pair of key tiles: numerics, microbench A/B
set -o pipefail
mkdir -p gpurun_out
K8SLLM_PREFILL_PAIRS=1 timeout -k 10 300 python -u -m pytest tests/test_ops_gpu.py -x -q -k "prefill" --timeout 120 --timeout-method thread > gpurun_out/pairs_tests.log 2>&1 || { tail -30 gpurun_out/pairs_tests.log; exit 1; }
tail -1 gpurun_out/pairs_tests.log
for r in 1 2; do
for p in 0 1; do
  K8SLLM_PREFILL_PAIRS=$p timeout -k 10 200 python tools/bench_prefill_attn.py --only v2 > gpurun_out/pairs_$p.jsonl 2>gpurun_out/pairs.err || { tail gpurun_out/pairs.err; exit 1; }
  K8SLLM_PREFILL_PAIRS=$p timeout -k 10 200 python tools/bench_prefill_attn.py --only v2 --seqs 4 --len 4000 >> gpurun_out/pairs_$p.jsonl 2>>gpurun_out/pairs.err || { tail gpurun_out/pairs.err; exit 1; }
  echo "pairs=$p"; cat gpurun_out/pairs_$p.jsonl
done
done
