# in-engine A/B: decode attention unsplit (default at batch 64) vs 2 splits + merge launch
# (ragged 1.2k-2.2k contexts: do more, smaller workgroups balance the tail?)
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
: > gpurun_out/split_ab.txt
for r in 1 2; do for sp in 0 2; do
  if [ $sp = 0 ]; then unset K8SLLM_DECODE_SPLITS; else export K8SLLM_DECODE_SPLITS=$sp; fi
  timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/pt_sp -o run -- python3 bench.py --steps 1 --warmup 1 > gpurun_out/pt_sp.log 2>&1 || { tail -30 gpurun_out/pt_sp.log; exit 1; }
  f=$(find gpurun_out/pt_sp -name "*results.db" | head -1)
  python3 - "$f" "$sp" "$r" >> gpurun_out/split_ab.txt <<'PY'
import sqlite3, sys, collections
c = sqlite3.connect(sys.argv[1])
agg = collections.defaultdict(list)
for name, s, e in c.execute("select name, start, end from kernels"):
    if "paged_decode" in name:
        agg[name.split("(")[0][-60:]].append(e - s)
print(f"splits={sys.argv[2]} round={sys.argv[3]} " + " | ".join(f"{k}: {sum(v)/len(v)/1e3:.2f} us x{len(v)} total {sum(v)/1e6:.1f} ms" for k, v in agg.items()))
PY
  rm -rf gpurun_out/pt_sp
done; done
cat gpurun_out/split_ab.txt
