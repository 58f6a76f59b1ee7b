# every BASELINE config on the current tree, one GPU.  PART=a: Mixtral (bench +
# kernel trace); PART=c: the 70B TP=1 proxy; PART=b: podcomm, latency, production 2000-token, Poisson.
set -o pipefail
mkdir -p gpurun_out
part=${1:-a}
b() {  # tag, limit, bench args...
  local tag=$1 lim=$2; shift 2
  timeout -k 10 $lim python bench.py --out gpurun_out/cfg_$tag.json "$@" > gpurun_out/cfg_$tag.log 2>&1 \
    || { tail -20 gpurun_out/cfg_$tag.log; exit 1; }
  cut -c1-260 gpurun_out/cfg_$tag.json
}
if [ "$part" = a ]; then
  b mixtral 600 --model mixtral-8x7b --steps 3 --warmup 1
  bash scripts/gpu/run.sh prof mixtral --model mixtral-8x7b > gpurun_out/prof_mixtral_out.txt 2>&1 \
    || { tail -20 gpurun_out/prof_mixtral_out.txt; exit 1; }
  head -3 gpurun_out/prof_mixtral_steps.txt; grep -c "Cijk_" gpurun_out/prof_mixtral_summary.md || true
elif [ "$part" = c ]; then
  b llama70b_tp1 700 --model llama-3-70b --steps 2 --warmup 1
else
  b podcomm 400 --path podcomm --steps 3 --warmup 1
  b latency 300 --mode latency --steps 5 --warmup 1
  b prod2000 500 --production --max-new-tokens 2000 --steps 2 --warmup 1
  b poisson16 400 --mode poisson --rate 16 --steps 2 --warmup 1
fi
