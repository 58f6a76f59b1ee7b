"""Does smoke() catch a wrong kernel?  Runs __graft_entry__.smoke() once with a one-line fault
injected into the decode attention (its output negated - the kind of error a broken kernel
that still emits token ids would make) and expects the numeric check to fail.

    python tools/smoke_fault.py        # exit 0 = the fault was caught, 1 = smoke passed anyway
"""
from __future__ import annotations

import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main() -> int:
    import __graft_entry__ as g
    from k8s_llm_monitor_amd import ops

    orig = ops.paged_decode_fused

    def faulty(*a, **k):
        out = orig(*a, **k)
        return out.neg_()  # the injected fault

    ops.paged_decode_fused = faulty
    try:
        g.smoke()
    except AssertionError as e:
        print(f"smoke caught the injected fault: {e}")
        return 0
    print("smoke PASSED with a faulty decode kernel")
    return 1


if __name__ == "__main__":
    sys.exit(main())
