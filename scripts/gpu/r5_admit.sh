# admission window A/B on the headline: the first prefill of a wave waits for a full 16k-token
# step or admit_window_ms (default 20); a shorter window starts a partial first step while the rest
# of the burst is still arriving.  Interleaved, 2 rounds.
set -o pipefail
mkdir -p gpurun_out
for i in 1 2; do
  for w in 20 4; do
    timeout -k 10 300 python bench.py --steps 5 --warmup 2 --admit-window-ms $w --out gpurun_out/adm_${w}_$i.json \
      > gpurun_out/adm_${w}_$i.log 2>&1 || { tail -20 gpurun_out/adm_${w}_$i.log; exit 1; }
    python3 -c "import json;d=json.load(open('gpurun_out/adm_${w}_$i.json'));print('window $w round $i', d['value'], d['p50_latency_ms'], d['prefill_steps'])"
  done
done
