# GPU idle gaps in the headline wave: kernel trace, then gaps > 50 us between consecutive kernels
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 400 rocprofv3 --kernel-trace -d gpurun_out/prof_g -o run -- python3 bench.py --steps 2 --warmup 1 > gpurun_out/prof_g.log 2>&1 || { tail -30 gpurun_out/prof_g.log; exit 1; }
f=$(find gpurun_out/prof_g -name "*results.db" | head -1)
python3 - "$f" > gpurun_out/gaps.txt <<'PY'
import sqlite3, sys, collections
c = sqlite3.connect(sys.argv[1])
rows = c.execute("select name, start, end from kernels order by start").fetchall()
t0, t1 = rows[0][1], rows[-1][2]
busy_end = rows[0][2]
# the timed region: the last two waves (~2.75 s each) end at the last kernel
win0 = t1 - int(5.6e9)
gaps = []
for (n0, s0, e0), (n1, s1, e1) in zip(rows, rows[1:]):
    if s1 < win0:
        busy_end = max(busy_end, e0)
        continue
    busy_end = max(busy_end, e0)
    g = s1 - busy_end
    if g > 50_000:
        gaps.append((g, n0.split("(")[0][-40:], n1.split("(")[0][-40:], s1))
tot = sum(g for g, *_ in gaps)
print(f"last 5.6 s of {(t1 - t0) / 1e6:.1f} ms span: gaps>50us: {len(gaps)} totalling {tot / 1e6:.1f} ms")
small = 0
be = rows[0][2]
for (n0, s0, e0), (n1, s1, e1) in zip(rows, rows[1:]):
    be = max(be, e0)
    if s1 >= win0 and 0 < s1 - be <= 50_000:
        small += s1 - be
print(f"gaps <= 50 us in the window: {small / 1e6:.1f} ms")
by = collections.Counter()
cnt = collections.Counter()
for g, a, b, s in gaps:
    by[(a, b)] += g
    cnt[(a, b)] += 1
for (a, b), g in by.most_common(15):
    print(f"{g / 1e6:8.2f} ms  x{cnt[(a, b)]:4d}  after {a}  before {b}")
big = sorted(gaps, reverse=True)[:10]
print("largest:", [(round(g / 1e6, 2), a, b) for g, a, b, s in big])
PY
cat gpurun_out/gaps.txt
rm -rf gpurun_out/prof_g
