# round 6: o / down decode GEMMs with 4 split-K slabs instead of 8 (half the slab bytes the
# add_norm_partial launches read) - whole decode step A/B in one engine
set -o pipefail
mkdir -p gpurun_out
for sw in split4 split4o split4d; do
  timeout -k 10 400 python -u tools/bench_decode_step.py --switch $sw --rows 64,16 --rounds 3 --tokens 96 \
    > gpurun_out/dstep_$sw.jsonl 2> gpurun_out/dstep_$sw.err || { tail -20 gpurun_out/dstep_$sw.err; exit 1; }
  grep on_median gpurun_out/dstep_$sw.jsonl
done
