# paged decode with double-buffered 32-token chunks: numerics, isolated sweep, GPU suite, headline
set -o pipefail
mkdir -p gpurun_out
true
tail -2 gpurun_out/gputests_h.log
for a in "64 1800" "64 4000" "8 1800" "1 1800"; do PYTHONPATH=. timeout -k 10 120 python tools/bench_decode.py $a >> gpurun_out/decode_db.txt 2>gpurun_out/decode_db.err || { tail gpurun_out/decode_db.err; exit 1; }; done
cat gpurun_out/decode_db.txt
timeout -k 10 300 python bench.py --steps 5 --warmup 2 > gpurun_out/bench_h.log 2>&1 || { tail -20 gpurun_out/bench_h.log; exit 1; }
tail -1 gpurun_out/bench_h.log
