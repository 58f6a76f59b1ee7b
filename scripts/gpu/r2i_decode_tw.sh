# paged decode: 32-token double-buffered vs 64-token single-buffered, isolated and in the engine
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_ops_gpu.py -x -q -k "paged or decode" --timeout 120 --timeout-method thread > gpurun_out/dec_tests.log 2>&1 || { tail -30 gpurun_out/dec_tests.log; exit 1; }
tail -1 gpurun_out/dec_tests.log
: > gpurun_out/decode_tw.txt
for tw in 32 64; do for a in "64 1800" "8 1800" "1 1800"; do echo "TW=$tw $a" >> gpurun_out/decode_tw.txt; K8SLLM_DECODE_TW=$tw PYTHONPATH=. timeout -k 10 120 python tools/bench_decode.py $a >> gpurun_out/decode_tw.txt 2>gpurun_out/decode_tw.err || { tail gpurun_out/decode_tw.err; exit 1; }; done; done
cat gpurun_out/decode_tw.txt
for tw in 32 64; do
K8SLLM_DECODE_TW=$tw timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_tw$tw -o run -- python3 bench.py --steps 2 --warmup 1 > gpurun_out/prof_tw$tw.log 2>&1 || { tail -30 gpurun_out/prof_tw$tw.log; exit 1; }
f=$(find gpurun_out/prof_tw$tw -name "*results.db" | head -1)
python3 tools/rocpd_summary.py $f --top 12 --title "TW=$tw" > gpurun_out/prof_tw${tw}_summary.md
grep -E "paged_decode|Total|total" gpurun_out/prof_tw${tw}_summary.md | head -5
done
