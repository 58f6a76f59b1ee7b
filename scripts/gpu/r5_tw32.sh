# small-batch paged decode: 128-token chunks (TW 32, double-buffered) vs the 256-token single-buffered
# form the launcher picks for split grids - more, lighter workgroups per (sequence, kv head)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u tools/bench_decode_step.py --switch tw32 --rows 1,2,4,8,16 --rounds 3 --tokens 64 \
  > gpurun_out/tw_ab.jsonl 2> gpurun_out/tw_ab.err || { tail -20 gpurun_out/tw_ab.err; exit 1; }
grep on_median gpurun_out/tw_ab.jsonl
