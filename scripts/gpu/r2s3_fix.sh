# 2-wave deferred-norm fix: targeted tests, the LM-head microbench, full GPU suite, headline bench
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_skinny_rm_gpu.py tests/test_real_shape_gpu.py -x -v --timeout 240 --timeout-method thread > gpurun_out/fix_tests.log 2>&1 || { tail -40 gpurun_out/fix_tests.log; exit 1; }
tail -3 gpurun_out/fix_tests.log
timeout -k 10 200 python -u tools/bench_lm_head.py --ms 1,16,32,64 > gpurun_out/lm_head_fixed.jsonl 2>/dev/null || exit 1
cat gpurun_out/lm_head_fixed.jsonl
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gputests.log 2>&1 || { tail -40 gpurun_out/gputests.log; exit 1; }
tail -2 gpurun_out/gputests.log
timeout -k 10 300 python bench.py --steps 5 --warmup 2 > gpurun_out/bench_fix.log 2>&1 || { tail -20 gpurun_out/bench_fix.log; exit 1; }
tail -1 gpurun_out/bench_fix.log | cut -c1-400
