# kernel trace of the headline bench with the final round-2 tree
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_s3 -o run -- python3 bench.py --steps 2 --warmup 1 > gpurun_out/prof_s3.log 2>&1 || { tail -30 gpurun_out/prof_s3.log; exit 1; }
tail -1 gpurun_out/prof_s3.log | cut -c1-200
f=$(find gpurun_out/prof_s3 -name "*results.db" | head -1)
python3 tools/rocpd_summary.py $f --top 40 --title "session-3 final headline bench (deferred-norm fix, DMA/MFMA interleave, 16-byte decode V loads, span-ordered flash q-blocks)" > gpurun_out/prof_s3_summary.md
python3 - "$f" > gpurun_out/prof_s3_steps.txt <<'PY'
import sqlite3, sys
c = sqlite3.connect(sys.argv[1])
rows = c.execute("select name, start, end from kernels order by start").fetchall()
# decode steps: sample_final marks the end of every step; sum kernel time between consecutive markers
marks = [i for i, r in enumerate(rows) if 'sample_final' in r[0]]
spans = []
for a, b in zip(marks, marks[1:]):
    ks = rows[a + 1:b + 1]
    if any('paged_decode_kernel' in r[0] for r in ks) and not any('flash_prefill' in r[0] for r in ks):
        busy = sum(r[2] - r[1] for r in ks)
        wall = ks[-1][2] - rows[a][2]
        spans.append((busy, wall))
spans.sort()
if spans:
    n = len(spans)
    med = spans[n // 2]
    print(f"decode steps {n}: median kernel-busy {med[0]/1e6:.3f} ms, wall {med[1]/1e6:.3f} ms (between step ends)")
    print(f"mean busy {sum(s[0] for s in spans)/n/1e6:.3f} ms, mean wall {sum(s[1] for s in spans)/n/1e6:.3f} ms")
PY
cat gpurun_out/prof_s3_steps.txt
rm -rf gpurun_out/prof_s3
timeout -k 10 300 python bench.py --steps 5 --warmup 2 --out gpurun_out/bench_s3_final.json > gpurun_out/bench_s3_final.log 2>&1 || { tail -20 gpurun_out/bench_s3_final.log; exit 1; }
cut -c1-200 gpurun_out/bench_s3_final.json
