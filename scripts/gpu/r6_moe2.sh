# round 6: Mixtral-8x7B TP=1 one layout vs two, second interleaved pair (two, one, two, one)
set -o pipefail
mkdir -p gpurun_out
for r in 2 3; do
  for lay in two one; do
    timeout -k 10 500 python bench.py --model mixtral-8x7b --steps 3 --warmup 1 --layout $lay --out gpurun_out/mx_${lay}_$r.json \
      > gpurun_out/mx_${lay}_$r.log 2>&1 || { tail -20 gpurun_out/mx_${lay}_$r.log; exit 1; }
    python3 -c "import json;d=json.load(open('gpurun_out/mx_${lay}_$r.json'));print('$lay $r', d['value'], d['config']['resident_weight_gb_per_rank'])"
  done
done
