#!/usr/bin/env python
"""Host cost of the headline's HTTP path, without a GPU: one closed-loop wave of N concurrent
``POST /api/v1/query`` through the real server stack (MonitorApp, AnalysisService with the
cluster-context builder, LocalEngineBackend) against an instant engine stand-in that answers every
request at once when the whole wave has arrived - the shape of a bench.py wave, whose answers all
finish on the same decode step.  Clients run in the out-of-process load generator, as in bench.py.

    python tools/bench_http_wave.py [--n 64 --waves 6 --answer-tokens 256]

Prints per wave: arrival span (first -> last submit), the resolve -> last response span, and the
wall time of the whole wave (what the wave boundary costs the GPU in bench.py)."""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys
import threading
import time
from concurrent.futures import Future

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


class _Seq:
    def __init__(self, n_prompt: int, out: list, t0: float):
        self.prompt_ids = [0] * n_prompt
        self.output_ids = out
        self.t_arrival = t0
        self.t_first_token = t0
        self.t_finish = None
        self.n_preemptions = 0
        self.finish_reason = "length"

    def timings(self) -> dict:
        from k8s_llm_monitor_amd.engine.sequence import Sequence

        return Sequence.timings(self)


class InstantService:
    """EngineService stand-in: collects a wave's submits, answers them together."""

    def __init__(self, n: int, answer_tokens: int):
        from types import SimpleNamespace

        from k8s_llm_monitor_amd.engine.tokenizer import tokenizer_for
        from k8s_llm_monitor_amd.models.config import get_config

        mc = get_config("llama-3-8b")
        self.engine = SimpleNamespace(model_cfg=mc, tokenizer=tokenizer_for(mc),
                                      cfg=SimpleNamespace(max_model_len=8192))
        self.n, self.answer = n, [1000 + (i * 37) % 20000 for i in range(answer_tokens)]
        self.lock = threading.Lock()
        self.pending: list = []
        self.t_submit: list = []
        self.t_resolve = 0.0
        self.healthy = True
        self.engine.tokenizer.decode(self.answer)  # build the decode table outside the clock

    def submit(self, prompt, params, request_id=None, deadline=None, on_tokens=None):
        ids = self.engine.tokenizer.encode(prompt)
        fut: Future = Future()
        with self.lock:
            self.t_submit.append(time.perf_counter())
            self.pending.append((fut, len(ids)))
            if len(self.pending) < self.n:
                return fut
            batch, self.pending = self.pending, []
        self.t_resolve = time.perf_counter()
        text = self.engine.tokenizer.decode(self.answer)
        for f, n_prompt in batch:
            f.set_result((text, _Seq(n_prompt, list(self.answer), self.t_resolve)))
        return fut

    def cancel(self, fut) -> None:
        pass

    def stats(self) -> dict:
        return {}


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=64)
    ap.add_argument("--waves", type=int, default=6)
    ap.add_argument("--answer-tokens", type=int, default=256)
    ap.add_argument("--switch-ms", type=float, default=0.0, help="sys.setswitchinterval for the server process")
    a = ap.parse_args()
    if a.switch_ms > 0:
        sys.setswitchinterval(a.switch_ms * 1e-3)
    from k8s_llm_monitor_amd.monitor.loadgen import LoadGen

    lg = LoadGen(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from k8s_llm_monitor_amd.llm.synthetic import synthetic_context
    from k8s_llm_monitor_amd.monitor.app import build_app_for_bench

    svc = InstantService(a.n, a.answer_tokens)
    srv, port = build_app_for_bench(svc)
    items = [synthetic_context(s)[::-1] for s in range(a.n)]
    lg.stage("w", items)
    walls, spans, tails = [], [], []
    try:
        for w in range(a.waves):
            svc.t_submit = []
            t0 = time.perf_counter()
            lg.post_queries(port, None, a.answer_tokens, slim=True, staged="w")
            t1 = time.perf_counter()
            walls.append((t1 - t0) * 1e3)
            spans.append((max(svc.t_submit) - min(svc.t_submit)) * 1e3)
            tails.append((t1 - svc.t_resolve) * 1e3)
            print(json.dumps({"wave": w, "wall_ms": round(walls[-1], 2), "arrival_span_ms": round(spans[-1], 2),
                              "first_submit_ms": round((min(svc.t_submit) - t0) * 1e3, 2),
                              "resolve_to_all_answers_ms": round(tails[-1], 2)}), flush=True)
    finally:
        lg.close()
        srv.shutdown()
    med = statistics.median
    print(json.dumps({"n": a.n, "wall_ms_median": round(med(walls[1:]), 2),
                      "arrival_span_ms_median": round(med(spans[1:]), 2),
                      "resolve_to_all_answers_ms_median": round(med(tails[1:]), 2)}), flush=True)


if __name__ == "__main__":
    main()
