set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gemm_decode_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t_dec.log 2>&1; rc=$?; tail -15 gpurun_out/t_dec.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python tools/bench_decode_gemm.py --rounds 3 > gpurun_out/dec_sweep.jsonl 2> gpurun_out/dec_sweep.err || { tail -20 gpurun_out/dec_sweep.err; exit 1; }
grep '"us"' gpurun_out/dec_sweep.jsonl | python3 -c "
import sys,json
for l in sys.stdin:
    d=json.loads(l); print(d['op'],d['M'],d['impl'],d['us'],d['TBps'])
"
