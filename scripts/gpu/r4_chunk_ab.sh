# prefill chunk budget A/B on the headline: 16k (default) vs 32k tokens per prefill step, interleaved
set -o pipefail
mkdir -p gpurun_out
for r in 1 2; do
  for c in 16384 32768; do
    timeout -k 10 300 python bench.py --steps 4 --warmup 2 --max-prefill-tokens $c --out gpurun_out/bench_chunk${c}_$r.json > gpurun_out/bench_chunk${c}_$r.log 2>&1 || { tail -20 gpurun_out/bench_chunk${c}_$r.log; exit 1; }
    echo "chunk=$c $r $(cut -c80-110 gpurun_out/bench_chunk${c}_$r.json)"
  done
done
