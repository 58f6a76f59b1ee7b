# interpreter thread-switch interval A/B (engine thread vs 64 HTTP handler threads during a wave's
# arrival burst): default 5 ms vs 1 ms vs 0.5 ms, interleaved, with the host trace
set -o pipefail
mkdir -p gpurun_out
for i in 1 2; do
  for sw in 5 1 0.5; do
    BENCH_SWITCH_MS=$sw K8SLLM_TRACE=1 timeout -k 10 300 python bench.py --steps 5 --warmup 2 --out gpurun_out/sw_${sw}_$i.json \
      > gpurun_out/sw_${sw}_$i.log 2>&1 || { tail -20 gpurun_out/sw_${sw}_$i.log; exit 1; }
    python3 -c "import json;d=json.load(open('gpurun_out/sw_${sw}_$i.json'));print('switch $sw round $i', d['value'])"
    grep "first prefill launched" gpurun_out/sw_${sw}_$i.log | sed 's/.*first add -> first prefill [0-9.]* ms, //' | tr '\n' ' '; echo
  done
done
