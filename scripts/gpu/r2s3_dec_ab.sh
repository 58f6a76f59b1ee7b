# same-box A/B of paged decode: 16-byte V loads (this tree) vs two 8-byte loads (_ab_old = previous commit)
set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/dec_ab.txt
for r in 1 2; do
  for t in new old; do
    d=.; [ $t = old ] && d=_ab_old
    for cfg in "64 1800" "1 2000"; do
      (cd $d && PYTHONPATH=. timeout -k 10 120 python tools/bench_decode.py $cfg 2>/dev/null) | grep -E "S= *(1|16|32) " | sed "s/^/$t r$r /" >> gpurun_out/dec_ab.txt || exit 1
    done
  done
done
cat gpurun_out/dec_ab.txt
