# deep-ring decode GEMM configs (microbench), then the full GPU suite + smoke + headline, then the
# headline kernel trace
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python tools/bench_decode_gemm.py --ms 64,32 --ops qkv,o,down --rounds 3 \
  --cfgs "qkv:4,1,8,8|8,1,8,16|4,1,8,32;o:8,1,8,8|8,1,8,16|4,1,8,32;down:8,1,8,8|14,1,8,16|14,1,8,32|7,1,8,32" \
  > gpurun_out/dec_deep.jsonl 2> gpurun_out/dec_deep.err || { tail -20 gpurun_out/dec_deep.err; exit 1; }
grep '"us"' gpurun_out/dec_deep.jsonl | cut -c1-120
bash scripts/gpu/run.sh suite && bash scripts/gpu/run.sh prof fused1
