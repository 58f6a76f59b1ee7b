#!/usr/bin/env python
"""Decode-step A/B inside ONE engine (one box, interleaved rounds): the headline model's real
decode hipGraph at 64 rows and ~1.7k-token contexts, timed by the engine's own GPU events
(``LLMEngine.step_samples``: back-to-back decode steps), with a path switch flipped and the
graphs re-captured between phases.

    python tools/bench_decode_step.py --switch rc [--rounds 3 --tokens 96]

Switches: ``rc`` - the row-complete o projection, on in every bucket vs off; ``merge`` - the
attention's split partials merged in-launch (ops.DECODE_MERGE) vs a paged_decode_reduce launch (CausalLM.set_decode_fusion).  (Round 5
also A/B'd write-through (sc1) epilogue stores in gemm_decode.hip with this tool: 6.107 vs 6.068
ms per step, slower - profiles/r05/decode_step_writethrough_ab.jsonl.  Round 6: ``split4*`` - o /
down on 4 split-K slabs instead of 8 (half the bytes add_norm_partial reads) - 6.02 vs 5.93 ms at 64
rows, 3.78 vs 3.75 at 16: slower, DEC_TABLE unchanged; profiles/r06/decode_step_split4_ab.jsonl.)
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

SWITCHES = {"rc": lambda m, on: m.set_decode_fusion(rc=on),
            "merge": lambda m, on: setattr(_ops(), "DECODE_MERGE", on is not False),
            "tw32": lambda m, on: _ops().native().decode_tw_force(32 if on else 0),
            # fewer split-K slabs for o / down (4 splits x 64 column groups of 4-wave workgroups
            # instead of 8 x 32 of 8-wave ones): half the slab bytes add_norm_partial reads
            "split4": lambda m, on: _dec_table(on, {(4096, 4096, 0): (4, 1, 4, 16), (4096, 14336, 0): (4, 1, 4, 16)}),
            "split4o": lambda m, on: _dec_table(on, {(4096, 4096, 0): (4, 1, 4, 16)}),
            "split4d": lambda m, on: _dec_table(on, {(4096, 14336, 0): (4, 1, 4, 16)})}
_DEC_DEFAULT: dict = {}


def _dec_table(on, alt: dict) -> None:
    t = _ops().DEC_TABLE
    for k, v in alt.items():
        _DEC_DEFAULT.setdefault(k, t.get(k))
        t[k] = v if on else _DEC_DEFAULT[k]


def _ops():
    from k8s_llm_monitor_amd import ops
    return ops


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--switch", default="rc", choices=sorted(SWITCHES))
    ap.add_argument("--model", default="llama-3-8b")
    ap.add_argument("--rows", default="64", help="decode batch; a comma list runs each in turn")
    ap.add_argument("--ctx", type=int, default=1700)
    ap.add_argument("--tokens", type=int, default=96)
    ap.add_argument("--rounds", type=int, default=3)
    a = ap.parse_args()
    from k8s_llm_monitor_amd.engine import EngineConfig, LLMEngine, SamplingParams

    rows_list = [int(r) for r in a.rows.split(",")]
    eng = LLMEngine(EngineConfig(model=a.model, max_num_seqs=max(rows_list), max_model_len=4096, kv_cache_gb=48.0,
                                 seed=1), device="cuda")
    eng.warmup()
    g = torch.Generator().manual_seed(5)
    sp = SamplingParams(max_tokens=a.tokens, temperature=0.0, ignore_eos=True)
    set_sw = SWITCHES[a.switch]
    for rows in rows_list:
        prompts = [torch.randint(100, 120000, (a.ctx + (i * 37) % 200,), generator=g).tolist() for i in range(rows)]
        res: dict = {True: [], False: []}
        for rnd in range(a.rounds):
            for on in (True, False):
                set_sw(eng.model, on)
                eng.runner.graphs.clear()
                eng.runner.capture_graphs()
                eng.step_samples.clear()
                eng.generate(prompts, sp)
                ms = [m for (n, m, _) in eng.step_samples if n == rows]
                med = statistics.median(ms) if ms else float("nan")
                res[on].append(med)
                print(json.dumps({"switch": a.switch, "rows": rows, "on": on, "round": rnd, "steps": len(ms),
                                  "median_step_ms": round(med, 4)}), flush=True)
        print(json.dumps({"switch": a.switch, "rows": rows, "on_ms": [round(x, 4) for x in res[True]],
                          "off_ms": [round(x, 4) for x in res[False]],
                          "on_median": round(statistics.median(res[True]), 4),
                          "off_median": round(statistics.median(res[False]), 4)}), flush=True)
    set_sw(eng.model, None)


if __name__ == "__main__":
    main()
