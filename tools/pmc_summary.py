"""Sum rocprofv3 --pmc counter results per kernel (counter_collection CSV) and print one JSON line
per kernel whose name contains --kernel.

    python tools/pmc_summary.py gpurun_out/pmc1 --kernel flash_prefill_paged_v2
"""
from __future__ import annotations

import argparse
import csv
import glob
import json
import os
from collections import defaultdict


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--kernel", default="")
    a = ap.parse_args()
    tot: dict = defaultdict(lambda: defaultdict(float))
    calls: dict = defaultdict(set)
    for f in glob.glob(os.path.join(a.dir, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                name = row.get("Kernel_Name", "")
                if a.kernel not in name:
                    continue
                key = name.split("(")[0][:80]
                tot[key][row["Counter_Name"]] += float(row["Counter_Value"])
                calls[key].add(row.get("Dispatch_Id", ""))
    for k, v in tot.items():
        print(json.dumps({"kernel": k, "dispatches": len(calls[k]), **{c: int(x) for c, x in sorted(v.items())}}))


if __name__ == "__main__":
    main()
