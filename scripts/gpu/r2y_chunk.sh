# prefill step token budget A/B (interleaved): 16384 (default) vs 32768 vs 24576
set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/chunk.jsonl
for r in 1 2; do
for mp in 16384 32768 24576; do
  timeout -k 10 200 python bench.py --steps 3 --warmup 1 --max-prefill-tokens $mp > gpurun_out/chunk_$mp.log 2>&1 || { tail -20 gpurun_out/chunk_$mp.log; exit 1; }
  echo "{\"max_prefill_tokens\": $mp, \"round\": $r, \"line\": $(tail -1 gpurun_out/chunk_$mp.log)}" >> gpurun_out/chunk.jsonl
  tail -1 gpurun_out/chunk_$mp.log | cut -c1-160
done
done
