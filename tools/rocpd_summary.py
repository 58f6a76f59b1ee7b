#!/usr/bin/env python
"""Summarise a rocprofv3 ``--kernel-trace`` SQLite database (``*_results.db``) as a markdown
table: per-kernel total / calls / average, sorted by total time.

    python tools/rocpd_summary.py gpurun_out/prof1/run_results.db [--top 30] [--title "..."]
"""
from __future__ import annotations

import argparse
import sqlite3


def summarise(db: str, top: int = 30) -> tuple[list[tuple], float]:
    c = sqlite3.connect(db)
    rows = c.execute(
        "select name, count(*), sum(duration), avg(duration), max(grid_x*grid_y*grid_z/"
        "(workgroup_x*workgroup_y*workgroup_z)), max(lds_size), max(vgpr_count), max(accum_vgpr_count) "
        "from kernels group by name order by sum(duration) desc").fetchall()
    total = sum(r[2] for r in rows)
    return rows[:top], total


def short(name: str, n: int = 90) -> str:
    name = name.replace("|", "/")
    return name if len(name) <= n else name[: n - 3] + "..."


def decode_steps(db: str) -> None:
    """Median kernel-busy time of pure decode steps (the sampler's final kernel ends every step)."""
    c = sqlite3.connect(db)
    rows = c.execute("select name, start, end from kernels order by start").fetchall()
    marks = [i for i, r in enumerate(rows) if "sample_final" in r[0]]
    spans = []
    for a, b in zip(marks, marks[1:]):
        ks = rows[a + 1:b + 1]
        if any("paged_decode" in r[0] for r in ks) and not any("flash_prefill" in r[0] for r in ks):
            spans.append((sum(r[2] - r[1] for r in ks), ks[-1][2] - rows[a][2]))
    spans.sort()
    if not spans:
        print("no pure decode steps found")
        return
    n = len(spans)
    med = spans[n // 2]
    print(f"decode steps {n}: median kernel-busy {med[0] / 1e6:.3f} ms, wall {med[1] / 1e6:.3f} ms (between step ends)")
    print(f"mean busy {sum(s[0] for s in spans) / n / 1e6:.3f} ms, mean wall {sum(s[1] for s in spans) / n / 1e6:.3f} ms")


def gaps(db: str, window_s: float = 5.4, min_us: float = 20.0) -> None:
    """GPU idle time in the last ``window_s`` seconds of the trace (the timed waves): total idle,
    idle gaps longer than ``min_us`` grouped by the kernels around them, and the busy fraction."""
    import collections

    c = sqlite3.connect(db)
    rows = c.execute("select name, start, end from kernels order by start").fetchall()
    t1 = max(r[2] for r in rows)
    win0 = t1 - int(window_s * 1e9)
    be, idle, small = rows[0][2], 0, 0
    by, cnt = collections.Counter(), collections.Counter()
    for (n0, s0, e0), (n1, s1, e1) in zip(rows, rows[1:]):
        be = max(be, e0)
        if s1 < win0 or s1 <= be:
            continue
        g = s1 - be
        idle += g
        if g > min_us * 1e3:
            k = (n0.split("(")[0][-45:], n1.split("(")[0][-45:])
            by[k] += g
            cnt[k] += 1
        else:
            small += g
    print(f"last {window_s:.1f} s: idle {idle / 1e6:.1f} ms ({100 * idle / (window_s * 1e9):.1f} %), "
          f"of which gaps <= {min_us:.0f} us {small / 1e6:.1f} ms")
    for (a, b), g in by.most_common(12):
        print(f"{g / 1e6:8.2f} ms  x{cnt[(a, b)]:5d}  after {a}  before {b}")
    # the kernels around the three largest gaps (start relative to the gap, duration)
    big = []
    be = rows[0][2]
    for i in range(1, len(rows)):
        be = max(be, rows[i - 1][2])
        if rows[i][1] >= win0 and rows[i][1] - be > min_us * 1e3:
            big.append((rows[i][1] - be, i, be))
    def show(g, i, gs, ctx=4):
        print(f"-- gap {g / 1e6:.2f} ms:")
        for j in range(max(0, i - ctx), min(len(rows), i + ctx)):
            n, st, en = rows[j]
            print(f"   {(st - gs) / 1e3:+10.1f} us  {(en - st) / 1e3:8.1f} us  {n.split('(')[0][-60:]}")

    for g, i, gs in sorted(big, reverse=True)[:3]:
        show(g, i, gs)
    # one example (the median-sized gap) of each of the four costliest (before, after) classes,
    # with more context: where a recurring host stall sits in the step sequence
    for (a, b), _ in by.most_common(4):
        ex = sorted((g, i, gs) for g, i, gs in big
                    if (rows[i - 1][0].split("(")[0][-45:], rows[i][0].split("(")[0][-45:]) == (a, b))
        if ex:
            print(f"== class {a} -> {b}: {len(ex)} gaps, median example")
            show(*ex[len(ex) // 2], ctx=8)


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--top", type=int, default=30)
    ap.add_argument("--title", default="")
    ap.add_argument("--decode-steps", action="store_true", help="print decode-step kernel-busy statistics only")
    ap.add_argument("--gaps", type=float, default=0.0, help="print GPU idle gaps of the last GAPS seconds only")
    a = ap.parse_args()
    if a.gaps > 0:
        gaps(a.db, a.gaps)
        return
    if a.decode_steps:
        decode_steps(a.db)
        return
    rows, total = summarise(a.db, a.top)
    if a.title:
        print(f"# {a.title}\n")
    print(f"GPU kernel time total: {total / 1e6:.1f} ms\n")
    print("| total ms | % | calls | avg us | WGs | LDS B | VGPR | AGPR | kernel |")
    print("|---|---|---|---|---|---|---|---|---|")
    for name, calls, tot, avg, wgs, lds, vgpr, agpr in rows:
        print(f"| {tot / 1e6:.1f} | {100 * tot / total:.2f} | {calls} | {avg / 1e3:.1f} | {wgs} | {lds} | {vgpr} | "
              f"{agpr} | `{short(name)}` |")


if __name__ == "__main__":
    main()
