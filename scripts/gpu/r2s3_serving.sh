# serving lines with the session-3 tree: poisson (open loop), batch-1 latency, production timeouts at max_tokens 2000
set -o pipefail
mkdir -p gpurun_out/s3_serving
b() { n=$1; shift; timeout -k 10 400 python bench.py "$@" --out gpurun_out/s3_serving/$n.json > gpurun_out/s3_serving/$n.log 2>&1 || { tail -20 gpurun_out/s3_serving/$n.log; exit 1; }; cut -c1-160 gpurun_out/s3_serving/$n.json; }
b pois12 --steps 2 --warmup 1 --mode poisson --rate 12 --batch 64
b lat256 --mode latency --steps 5 --warmup 1 --max-new-tokens 256
b lat2000 --mode latency --steps 2 --warmup 1 --max-new-tokens 2000 --production
b prod2000_b64 --steps 1 --warmup 1 --max-new-tokens 2000 --production
b prod2000_b32 --steps 1 --warmup 1 --batch 32 --max-new-tokens 2000 --production
b podcomm --path podcomm --steps 2 --warmup 1
