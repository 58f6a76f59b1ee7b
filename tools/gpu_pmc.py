"""rocprofv3 PMC passes around one command, summed per kernel (one JSON line per kernel and pass).

Each ``--pass`` is one rocprofv3 run (counters of one pass must fit the per-block slot limits:
8 SQ, 4 TCC, 4 TCP, 2 TA, 2 TD, 2 GRBM).  This driver never touches the GPU itself; rocprofv3 is
started as a child with the program right after ``--``.

    python tools/gpu_pmc.py --pass "SQ_WAVE_CYCLES GRBM_GUI_ACTIVE" --kernel gemm --out x.jsonl -- \\
        python3 tools/bench_gemm_tile.py --only qkv --rounds 1 --iters 4
"""
from __future__ import annotations

import argparse
import json
import os
import shutil
import subprocess
import sys
import tempfile

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--pass", dest="passes", action="append", required=True)
    ap.add_argument("--kernel", default="")
    ap.add_argument("--out", required=True)
    ap.add_argument("--timeout", type=int, default=120)
    ap.add_argument("cmd", nargs=argparse.REMAINDER)
    a = ap.parse_args()
    cmd = a.cmd[1:] if a.cmd and a.cmd[0] == "--" else a.cmd
    import csv
    import glob
    from collections import defaultdict

    for i, ctrs in enumerate(a.passes):
        d = tempfile.mkdtemp(prefix="pmc", dir=os.environ.get("TMPDIR", "/tmp"))
        r = subprocess.run(["timeout", "-s", "KILL", str(a.timeout), "rocprofv3", "--output-format", "csv", "--pmc",
                            *ctrs.split(), "-d", d, "-o", "run", "--", *cmd], capture_output=True, text=True)
        if r.returncode != 0:
            sys.stderr.write(r.stdout[-3000:] + r.stderr[-3000:])
            sys.exit(r.returncode)
        tot: dict = defaultdict(lambda: defaultdict(float))
        calls: dict = defaultdict(set)
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            with open(f) as fh:
                for row in csv.DictReader(fh):
                    name = row.get("Kernel_Name", "")
                    if a.kernel and a.kernel not in name:
                        continue
                    key = name.split("(")[0][:90]
                    tot[key][row["Counter_Name"]] += float(row["Counter_Value"])
                    calls[key].add(row.get("Dispatch_Id", ""))
        with open(a.out, "a") as fo:
            for k, v in tot.items():
                fo.write(json.dumps({"pass": i, "kernel": k, "dispatches": len(calls[k]),
                                     **{c: int(x) for c, x in sorted(v.items())}}) + "\n")
        shutil.rmtree(d, ignore_errors=True)


if __name__ == "__main__":
    main()
