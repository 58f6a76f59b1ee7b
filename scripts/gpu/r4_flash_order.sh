#!/bin/bash
# Paged flash prefill: q-block orders (work / seq) - numerics then timing.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_ops_gpu.py -k "flash_prefill" > gpurun_out/flash_order_tests.txt 2>&1 || { tail -30 gpurun_out/flash_order_tests.txt; exit 1; }
tail -3 gpurun_out/flash_order_tests.txt
for sh in "10 1609" "4 4000" "4 8000" "1 16000"; do
  set -- $sh
  PLAIN=0 timeout -k 10 120 python -u tools/bench_prefill_attn.py --seqs $1 --len $2 --orders seq >> gpurun_out/flash_order.jsonl || exit 1
done
cat gpurun_out/flash_order.jsonl
