"""Serving robustness (SURVEY.md §5 failure detection / admission control; VERDICT r1 items 3-5,
ADVICE r1): admission never crashes on prefix-cache hits, mixed prefill+decode steps keep decodes
running, overload is rejected with 503, deadlines truncate instead of 504, timed-out / cancelled
requests free their KV blocks, and a failing step does not end serving."""
import concurrent.futures as cf
import http.client
import json
import time

import pytest

from k8s_llm_monitor_amd.engine import (EngineConfig, EngineOverloaded, EngineService, EngineUnavailable, LLMEngine,
                                        SamplingParams)
from k8s_llm_monitor_amd.engine.block_manager import BlockManager
from k8s_llm_monitor_amd.engine.scheduler import Scheduler, SchedulerConfig
from k8s_llm_monitor_amd.engine.sequence import Sequence, SeqStatus


@pytest.mark.parametrize("native", [False, True])
def test_admission_counts_idle_prefix_hits_as_consumed(native):
    """prefix-cache hits parked in the LRU are counted in num_free, so
    can_allocate must charge them; the scheduler must never run a sequence without blocks."""
    bm = BlockManager(8, use_native=native)
    if native and not bm.native:
        pytest.skip("native runtime not built")
    s = Scheduler(SchedulerConfig(max_num_seqs=4, max_prefill_tokens=4096, mixed_prefill_tokens=0), bm)
    shared = list(range(1000, 1033))  # 33 tokens: 2 full blocks publishable
    a = Sequence(prompt_ids=shared + [1], params=SamplingParams())
    s.add(a)
    p = s.schedule()
    assert p.seqs == [a]
    s.chunk_done(a)
    s.finish(a, "stop")  # its 2 full prompt blocks stay cached (LRU), 1 block freed
    assert bm.stats()["evictable_blocks"] == 2
    r = Sequence(prompt_ids=list(range(90)), params=SamplingParams())  # 6 blocks
    s.add(r)
    s.schedule()
    s.chunk_done(r)
    assert bm.num_free == 2  # the 2 idle cached blocks
    c = Sequence(prompt_ids=shared + [7, 8], params=SamplingParams())  # hits 2 blocks, needs 1 more
    assert not bm.can_allocate(c)  # 2 free - 1 fresh - 2 idle hits < 0 (the old check said yes)
    s.add(c)
    plan = s.schedule()  # must not crash; c waits (decode of r instead)
    assert c in s.waiting and all(q.block_table for q in s.running)
    assert not plan.is_prefill and plan.seqs == [r]


def test_mixed_step_keeps_decodes_running_and_matches_unmixed():
    """A prompt arriving while another sequence decodes joins a mixed step (decode rows ride the
    prefill forward); greedy outputs equal those of an engine that stalls decodes for prefill."""
    prompts = ["集群状态概览: node-000 NotReady, payments-api CrashLoopBackOff " * 2, "why is coredns failing? " * 3]
    sp = SamplingParams(max_tokens=8, temperature=0.0, ignore_eos=True)
    outs = {}
    for mixed in (4096, 0):
        eng = LLMEngine(EngineConfig(model="llama-tiny", max_num_seqs=4, max_model_len=512, num_blocks=128,
                                     use_graphs=False, seed=7, dtype="float32", prefix_caching=False,
                                     mixed_prefill_tokens=mixed, max_prefill_tokens=32,
                                     max_decode_stall_steps=0), device="cpu")
        a = eng.add_request(prompts[0], sp)
        for _ in range(8):  # a is chunked over 3 prefill steps (pipelined: read back one step later)
            if a.prefilled:
                break
            eng.step()
        assert a.prefilled and len(a.output_ids) >= 1
        b = eng.add_request(prompts[1], sp)
        n_a = len(a.output_ids)
        eng.step()
        if mixed:  # a got a token in the same step that started b's prefill
            assert eng.counters["mixed_steps"] == 1 and len(a.output_ids) == n_a + 1 and b.num_computed > 0
        while not all(q.status == SeqStatus.FINISHED for q in (a, b)):
            eng.step()
        outs[mixed] = [a.output_ids, b.output_ids]
        assert eng.blocks.num_free == 128
    assert outs[4096] == outs[0]


def test_mixed_step_scheduler_plan():
    s = Scheduler(SchedulerConfig(max_num_seqs=4, max_prefill_tokens=64, mixed_prefill_tokens=16),
                  BlockManager(64, use_native=False))
    a = Sequence(prompt_ids=list(range(10)), params=SamplingParams())
    s.add(a)
    s.schedule()
    s.chunk_done(a)
    a.output_ids.append(5)
    b = Sequence(prompt_ids=list(range(40)), params=SamplingParams())
    s.add(b)
    p = s.schedule()
    assert p.is_mixed and p.decode == [a] and p.seqs == [b] and b.chunk == 16  # mixed budget caps the chunk


def test_burst_policy_prefill_first_with_bounded_decode_stall():
    """A prefill backlog larger than one step's budget (a burst) runs prefill-only steps while the
    ready decodes wait, at most max_decode_stall_steps in a row, then one mixed step runs them; a
    backlog that fits one step is mixed at once."""
    s = Scheduler(SchedulerConfig(max_num_seqs=8, max_prefill_tokens=16, mixed_prefill_tokens=16,
                                  max_decode_stall_steps=2), BlockManager(256, use_native=False))
    a = Sequence(prompt_ids=list(range(10)), params=SamplingParams())
    s.add(a)
    s.schedule()
    s.chunk_done(a)
    a.output_ids.append(5)
    for i in range(3):  # 3 x 20 distinct tokens of backlog against a 16-token step
        s.add(Sequence(prompt_ids=list(range(100 * (i + 1), 100 * (i + 1) + 20)), params=SamplingParams()))
    kinds = []
    for _ in range(4):
        p = s.schedule()
        kinds.append("mixed" if p.is_mixed else ("prefill" if p.is_prefill else "decode"))
        if p.is_prefill:
            for q in p.seqs:
                s.chunk_done(q)
    # backlog 60, 44 -> prefill-only (2 = the bound); 28 -> the bound forces a mixed step; 12 fits
    # one step -> mixed
    assert kinds == ["prefill", "prefill", "mixed", "mixed"], kinds
    # steady state: the backlog fits one step -> mixed immediately
    s2 = Scheduler(SchedulerConfig(max_num_seqs=8, max_prefill_tokens=64, mixed_prefill_tokens=64,
                                   max_decode_stall_steps=2), BlockManager(256, use_native=False))
    c = Sequence(prompt_ids=list(range(10)), params=SamplingParams())
    s2.add(c)
    s2.schedule()
    s2.chunk_done(c)
    c.output_ids.append(1)
    s2.add(Sequence(prompt_ids=list(range(100, 120)), params=SamplingParams()))
    assert s2.schedule().is_mixed


def _tiny_engine(**kw):
    cfg = dict(model="llama-tiny", max_num_seqs=4, max_model_len=1024, num_blocks=256, use_graphs=False, seed=1)
    cfg.update(kw)
    return LLMEngine(EngineConfig(**cfg), device="cpu")


def test_queue_bound_rejects_with_overloaded():
    eng = _tiny_engine(max_num_seqs=2)
    svc = EngineService(eng, max_queue=3)
    try:
        sp = SamplingParams(max_tokens=40, temperature=0.0, ignore_eos=True)
        futs = [svc.submit(f"pod-{i} OOMKilled", sp) for i in range(12)]
        res = []
        for f in futs:
            try:
                f.result(timeout=120)
                res.append("ok")
            except EngineOverloaded:
                res.append("busy")
        assert "busy" in res and "ok" in res
        assert svc.stats()["rejected"] == res.count("busy")
    finally:
        svc.close()
    assert eng.blocks.num_free == eng.runner.num_blocks


def test_deadline_truncates_and_frees_blocks():
    eng = _tiny_engine()
    svc = EngineService(eng)
    try:
        sp = SamplingParams(max_tokens=100000, temperature=0.0, ignore_eos=True)
        t0 = time.perf_counter()
        text, seq = svc.submit("why?", sp, deadline=time.perf_counter() + 0.5).result(timeout=60)
        assert seq.finish_reason == "deadline" and len(seq.output_ids) > 0
        assert time.perf_counter() - t0 < 5
        assert eng.counters["deadline_stops"] == 1
    finally:
        svc.close()
    assert eng.blocks.num_free == eng.runner.num_blocks


def test_cancel_frees_blocks():
    eng = _tiny_engine()
    svc = EngineService(eng)
    try:
        fut = svc.submit("pod crash", SamplingParams(max_tokens=100000, ignore_eos=True))
        while not eng.sched.running:
            time.sleep(0.01)
        assert svc.cancel(fut)
        for _ in range(500):
            if not eng.sched.running and not eng.sched.waiting:
                break
            time.sleep(0.01)
        assert svc.stats()["cancelled"] == 1
    finally:
        svc.close()
    assert eng.blocks.num_free == eng.runner.num_blocks


def test_step_failure_fails_only_inflight_then_unhealthy():
    eng = _tiny_engine()
    svc = EngineService(eng, max_failures=2)
    real = eng.runner.prefill_launch  # every prefill path (pipelined and mixed) goes through it
    boom = {"n": 1}

    def flaky(*a, **k):
        if boom["n"] > 0:
            boom["n"] -= 1
            raise RuntimeError("injected HIP fault")
        return real(*a, **k)

    eng.runner.prefill_launch = flaky
    sp = SamplingParams(max_tokens=3, temperature=0.0, ignore_eos=True)
    try:
        with pytest.raises(RuntimeError, match="injected"):
            svc.submit("first", sp).result(timeout=60)
        assert svc.healthy and eng.blocks.num_free == eng.runner.num_blocks
        text, seq = svc.submit("second", sp).result(timeout=60)  # serving continues
        assert len(seq.output_ids) == 3
        boom["n"] = 1
        with pytest.raises(RuntimeError):
            svc.submit("third", sp).result(timeout=60)
        assert not svc.healthy and svc.stats()["healthy"] is False
        with pytest.raises(EngineUnavailable):
            svc.submit("fourth", sp).result(timeout=5)
    finally:
        svc.close()


def _post(port, q, max_tokens, timeout=120):
    body = json.dumps({"question": q, "max_tokens": max_tokens, "ignore_eos": True,
                       "context": {"cluster_state": "node-001 CPU=93.1% [资源压力]"}}).encode()
    conn = http.client.HTTPConnection("127.0.0.1", port, timeout=timeout)
    conn.request("POST", "/api/v1/query", body, {"Content-Type": "application/json"})
    r = conn.getresponse()
    data = json.loads(r.read())
    conn.close()
    return r.status, data


def test_http_flood_sees_503_not_504_and_frees_kv():
    """VERDICT r1 'do this' #3: flood /api/v1/query past capacity under production-like timeouts:
    overload answers 503 {"status":"error"}, long answers are truncated at the deadline (200,
    finish_reason "deadline"), nothing answers 504, and the KV cache ends empty."""
    from k8s_llm_monitor_amd.monitor.app import build_app_for_bench

    eng = _tiny_engine(max_num_seqs=2)
    svc = EngineService(eng, max_queue=2)
    srv, port = build_app_for_bench(svc, write_timeout_s=3.0, llm_timeout_s=30.0)
    try:
        with cf.ThreadPoolExecutor(16) as ex:
            res = list(ex.map(lambda i: _post(port, f"q{i}", 100000), range(16)))
        codes = [c for c, _ in res]
        assert 504 not in codes
        assert 503 in codes and 200 in codes
        for c, d in res:
            if c == 503:
                assert d["status"] == "error"
            else:
                assert d["status"] == "success" and d["result"]["finish_reason"] == "deadline"
        conn = http.client.HTTPConnection("127.0.0.1", port, timeout=10)
        conn.request("GET", "/health")
        assert conn.getresponse().status == 200
    finally:
        srv.shutdown()
        svc.close()
    assert eng.blocks.num_free == eng.runner.num_blocks


def test_tpot_model_fit():
    from k8s_llm_monitor_amd.engine.engine import TpotModel

    m = TpotModel(alpha=1.0)
    assert m.estimate(4) is None
    m.record(8, 40.0)
    assert m.estimate(4) == 40.0 and m.estimate(16) == 80.0  # one size: flat below, proportional above
    m.record(1, 10.0)
    m.record(64, 280.0)
    assert abs(m.estimate(32) - (10.0 + 270.0 / 63 * 31)) < 2.0  # the line through the points
    assert m.estimate(0) >= 10.0


def test_deadline_feasible_admission_refuses_instead_of_truncating():
    """with a learned step time that makes only a few answers fit the deadline,
    the service starts only those (every one completes, none is deadline-truncated) and refuses
    the rest at once with EngineOverloaded (HTTP 503) instead of truncating them later."""
    eng = LLMEngine(EngineConfig(model="llama-tiny", max_num_seqs=8, max_model_len=512, num_blocks=256,
                                 use_graphs=False, seed=3, dtype="float32", admit_window_ms=0), device="cpu")
    svc = EngineService(eng)
    try:
        # frozen step-time model: 20 ms at batch 1, +20 ms per extra row (CPU steps are far faster,
        # so admitted answers finish well inside their deadline)
        svc.tpot.record(1, 20.0)
        svc.tpot.record(8, 160.0)
        svc.tpot.record = lambda *a, **k: None
        sp = SamplingParams(max_tokens=24, temperature=0.0, ignore_eos=True)
        deadline = time.perf_counter() + 2.0  # 24 steps fit up to ~3 rows (24 * 60 ms * 1.05 = 1.5 s)
        futs = [svc.submit(f"pod-{i} CrashLoopBackOff, why?", sp, deadline=deadline) for i in range(8)]
        ok, refused = [], 0
        for f in futs:
            try:
                ok.append(f.result(timeout=60)[1])
            except EngineOverloaded:
                refused += 1
        assert 1 <= len(ok) <= 4 and refused == 8 - len(ok), (len(ok), refused)
        assert all(s.finish_reason == "length" and len(s.output_ids) == 24 for s in ok)
        assert svc.stats()["infeasible_rejected"] == refused
    finally:
        svc.close()


def _frozen_service(max_num_seqs=8):
    eng = LLMEngine(EngineConfig(model="llama-tiny", max_num_seqs=max_num_seqs, max_model_len=512, num_blocks=256,
                                 use_graphs=False, seed=3, dtype="float32", admit_window_ms=0), device="cpu")
    svc = EngineService(eng)
    return eng, svc


def test_admission_gate_preempted_sequence_resumes_and_does_not_freeze_admission():
    """a preempted sequence (answer tokens already generated) re-enters the waiting
    queue at the front; the gate must let it resume (sized by what is left, not its whole
    max_tokens) instead of refusing it and freezing every later admission until its deadline."""
    eng, svc = _frozen_service()
    try:
        svc.tpot.record(1, 20.0)
        svc.tpot.record(8, 160.0)
        sp = SamplingParams(max_tokens=100, temperature=0.0, ignore_eos=True)
        s = Sequence(prompt_ids=[5] * 10, params=sp, request_id="p", deadline=time.perf_counter() + 1.0)
        s.output_ids.extend([7] * 95)  # preempted after 95 tokens
        assert svc._admit_ok(s, 1)  # 100 x 20 ms would not fit 1 s: the remainder is not even asked
        assert svc._expected_rem(s) == 5
        fresh = Sequence(prompt_ids=[5] * 10, params=sp, request_id="f", deadline=time.perf_counter() + 1.0)
        assert not svc._admit_ok(fresh, 1)  # a fresh 100-token answer does not fit 1 s
    finally:
        svc.close()


def test_admission_gate_no_deadline_not_held_back_by_running_deadlines():
    eng, svc = _frozen_service()
    try:
        svc.tpot.record(1, 20.0)
        svc.tpot.record(8, 160.0)
        sp = SamplingParams(max_tokens=50, temperature=0.0, ignore_eos=True)
        run = Sequence(prompt_ids=[5] * 10, params=sp, request_id="r", deadline=time.perf_counter() + 1.2)
        eng.sched.running.append(run)  # 50 steps x ~20-40 ms: the running answer has almost no slack
        try:
            svc._prefill_tps = 1.0  # a prefill would take seconds: a deadline-bearing joiner is held
            timed = Sequence(prompt_ids=[5] * 10, params=sp, request_id="t", deadline=time.perf_counter() + 60)
            free = Sequence(prompt_ids=[5] * 10, params=sp, request_id="n")
            assert not svc._admit_ok(timed, 2)
            assert svc._admit_ok(free, 2)
        finally:
            eng.sched.running.remove(run)
    finally:
        svc.close()


def test_admission_budgets_eos_answers_by_observed_lengths():
    """answers that may stop on EOS are budgeted at the observed 90th-percentile answer
    length, not max_tokens: at the product default (max_tokens 2000) a short-answer workload is
    not refused as 'cannot finish'."""
    eng, svc = _frozen_service()
    try:
        svc.tpot.record(1, 6.0)
        svc.tpot.record(64, 7.0)
        eos = SamplingParams(max_tokens=2000, temperature=0.0)
        fixed = SamplingParams(max_tokens=2000, temperature=0.0, ignore_eos=True)
        dl = time.perf_counter() + 5.0
        a = Sequence(prompt_ids=[5] * 10, params=eos, request_id="a", deadline=dl)
        b = Sequence(prompt_ids=[5] * 10, params=fixed, request_id="b", deadline=dl)
        assert not svc._admit_ok(a, 8)  # no observations yet: budgeted at max_tokens (14 s > 5 s)
        for n in [120, 180, 250, 300, 90, 400, 220, 150] * 2:
            svc.answer_lens.record(n)
        svc._step_cache.clear()
        assert svc._expected_rem(a) == 400  # the 90th percentile of the 16 answers
        assert svc._admit_ok(a, 8)  # ~400 x 7 ms fits 5 s
        assert not svc._admit_ok(b, 8)  # ignore_eos: always the full 2000 tokens
    finally:
        svc.close()


def test_tpot_samples_from_engine_events_feed_the_model():
    eng, svc = _frozen_service()
    try:
        eng.step_samples.append((64, 5.9))
        eng.step_samples.append((64, 6.1))
        t0 = time.time()
        while eng.step_samples and time.time() - t0 < 10:  # the engine thread drains them
            time.sleep(0.01)
        time.sleep(0.1)
        assert svc._gpu_tpot and 5.9 <= svc.tpot.estimate(64) <= 6.1
    finally:
        svc.close()


def test_tpot_context_model_fit():
    """t(b, kv) = a + r*b + k*kv is recovered from (batch, context tokens, ms) samples; without a
    context spread (or with a poor fit) the batch-size-only model stays in charge."""
    from k8s_llm_monitor_amd.engine.engine import TpotModel

    m = TpotModel(alpha=1.0)
    for i in range(60):  # one batch size, context growing as the answers grow: no spread yet
        m.record(64, 3.0 + 0.02 * 64 + 0.021 * (100000 + 64 * 0) / 1000, kv=100000)
    assert m.kv_fit is None
    m = TpotModel(alpha=1.0)
    for b in (40, 64):
        for step in range(0, 2000, 20):
            kv = b * (1600 + step)
            m.record(b, 3.0 + 0.02 * b + 0.021 * kv / 1000, kv=kv)
    a, r, k, err = m.kv_fit
    assert abs(a - 3.0) < 0.05 and abs(r - 0.02) < 0.002 and abs(k - 0.021) < 0.001 and err < 1e-6
    # an answer that starts now at 64 rows x 1.6k context is priced at its own context, not at the
    # latest (longest-context) steps the per-batch EWMA follows
    assert abs(m.estimate(64, 64 * 1600) - (3.0 + 1.28 + 0.021 * 102.4)) < 0.01
    assert m.estimate(64) > m.estimate(64, 64 * 1600) + 2.0
    assert m.snapshot()["kv_fit"]["samples"] == 200


def test_admission_prices_answers_at_their_context():
    """The batch-size EWMA follows the latest, longest-context steps; the context-aware model
    prices a fresh answer at the mean context over its own life, so an answer that fits its
    deadline is admitted (production runs: 36 % refused with the EWMA alone)."""
    eng, svc = _frozen_service()
    try:
        for kv in range(1000, 9001, 100):  # 8 rows, step time 10 ms + 2 ms per 1k context tokens
            svc.tpot.record(8, 10.0 + 2.0 * kv / 1000, kv=kv)
        assert svc.tpot.kv_fit is not None and svc.tpot.estimate(8) > 27.0
        sp = SamplingParams(max_tokens=100, temperature=0.0, ignore_eos=True)
        s = Sequence(prompt_ids=[5] * 10, params=sp, request_id="c", deadline=time.perf_counter() + 2.0)
        # EWMA: 100 x 28 ms x 1.05 = 2.9 s > 2 s; at its context (10 + 8 x 50 tokens): ~1.2 s
        assert svc._admit_ok(s, 8)
        tight = Sequence(prompt_ids=[5] * 10, params=sp, request_id="t", deadline=time.perf_counter() + 1.0)
        assert not svc._admit_ok(tight, 8)
    finally:
        svc.close()


def test_admission_counts_the_burst_prefill_backlog():
    """Every answer of a burst waits for the whole burst's prefill before its first decode step:
    prompt tokens admitted but not yet computed delay a joiner's answer (and the running ones')."""
    eng, svc = _frozen_service()
    try:
        svc.tpot.record(1, 10.0)
        svc.tpot.record(8, 10.0)
        svc._prefill_tps = 1000.0  # 1k prompt tokens per second
        sp = SamplingParams(max_tokens=50, temperature=0.0, ignore_eos=True)
        joiner = Sequence(prompt_ids=[5] * 10, params=sp, request_id="j", deadline=time.perf_counter() + 1.0)
        assert svc._admit_ok(joiner, 2)  # 10 ms prefill + 50 x 10.5 ms fits 1 s
        queued = Sequence(prompt_ids=[5] * 800, params=sp, request_id="q")  # admitted, not yet prefilled
        eng.sched.running.append(queued)
        try:
            svc._step_cache.clear()
            assert svc._backlog_s() > 0.79
            assert not svc._admit_ok(joiner, 2)  # 0.8 s of backlog + 0.53 s no longer fits
            queued.num_computed = 800
            svc._step_cache.clear()
            assert svc._admit_ok(joiner, 2)
        finally:
            eng.sched.running.remove(queued)
    finally:
        svc.close()


def test_gather_burst_behind_a_full_prefill_step():
    """While a long enough prefill-only step runs on the GPU, the service keeps collecting a
    burst's arrivals before planning the next (pipelined) prefill step - but only when that step
    would not be full, no decode step is in flight, a sequence slot is free and the wait is hidden
    (a GPU device, the step's estimated time covers the window).  (A stand-in engine: the
    condition reads only this state.)"""
    import types

    cap = 64
    backlog = [0]
    sched = types.SimpleNamespace(running=[], cfg=types.SimpleNamespace(max_num_seqs=8),
                                  prefill_backlog=lambda: backlog[0])
    eng = types.SimpleNamespace(_pf_inflight=None, _inflight=None, sched=sched,
                                cfg=types.SimpleNamespace(admit_window_ms=20.0, max_prefill_tokens=cap),
                                device=types.SimpleNamespace(type="cpu"))
    svc = types.SimpleNamespace(engine=eng, _prefill_tps=None)
    ok = lambda: EngineService._gather_ok(svc)  # noqa: E731
    full = types.SimpleNamespace(chunks=[cap])
    assert not ok()  # nothing in flight
    eng._pf_inflight = (full, None, 1)
    assert not ok()  # CPU: a launched step has already run
    eng.device.type = "cuda"
    assert ok()  # a full step in flight, nothing queued behind it
    eng._pf_inflight = (types.SimpleNamespace(chunks=[cap // 4]), None, 1)
    assert not ok()  # a small step in flight: the wait would not be hidden
    svc._prefill_tps = 400.0  # measured: 16 tokens take 40 ms >= the 20 ms window
    assert ok()
    svc._prefill_tps = 4000.0  # 4 ms: not hidden
    assert not ok()
    svc._prefill_tps = None
    eng._pf_inflight = (full, None, 1)
    eng._inflight = ([], None)
    assert not ok()  # a decode step in flight
    eng._inflight = None
    backlog[0] = cap
    assert not ok()  # the next step is already full
    backlog[0] = 0
    sched.running = [None] * 8
    assert not ok()  # no free sequence slot: more arrivals could not join the next step
    eng.cfg.admit_window_ms = 0.0
    sched.running = []
    assert not ok()  # coalescing disabled
