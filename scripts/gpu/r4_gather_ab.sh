# Headline A/B: gathering a burst behind a running full prefill step (K8SLLM_PREFILL_GATHER) -
# a traced run of each (the prefill step splits), then interleaved plain runs
set -o pipefail
mkdir -p gpurun_out
for g in 1 0; do
  K8SLLM_PREFILL_GATHER=$g K8SLLM_TRACE=1 timeout -k 10 300 python bench.py --steps 3 --warmup 1 --out gpurun_out/bench_gtrace$g.json > gpurun_out/bench_gtrace$g.log 2>&1 || { tail -20 gpurun_out/bench_gtrace$g.log; exit 1; }
  grep "trace\] prefill" gpurun_out/bench_gtrace$g.log | head -24 > gpurun_out/gather_prefill_steps_$g.txt
done
for r in 1 2; do
  for g in 1 0; do
    K8SLLM_PREFILL_GATHER=$g timeout -k 10 300 python bench.py --steps 5 --warmup 2 --out gpurun_out/bench_gather${g}_$r.json > gpurun_out/bench_gather${g}_$r.log 2>&1 || { tail -20 gpurun_out/bench_gather${g}_$r.log; exit 1; }
    python3 -c "import json;d=json.load(open('gpurun_out/bench_gather${g}_$r.json'));print('gather=$g run $r', d['value'], d['ms_per_step'])"
  done
done
