"""Engine correctness: paged-KV incremental decode must reproduce a full recompute of the same
sequence (the cache, RoPE positions, block tables and scheduler bookkeeping all feed this)."""
import pytest
import torch

from k8s_llm_monitor_amd.engine import EngineConfig, LLMEngine, SamplingParams
from k8s_llm_monitor_amd.engine.sequence import SeqStatus
from k8s_llm_monitor_amd.models import AttnMeta


def _full_logits(model, ids, device):
    n = len(ids)
    t = torch.tensor(ids, dtype=torch.int32, device=device)
    meta = AttnMeta(is_prefill=True, positions=torch.arange(n, dtype=torch.int32, device=device),
                    slot_mapping=torch.full((n,), -1, dtype=torch.int32, device=device),
                    cu_seqlens=torch.tensor([0, n], dtype=torch.int32, device=device),
                    logits_idx=torch.tensor([n - 1], device=device))
    return model.forward(t, meta, None)[0].float()


def _check_greedy_consistency(eng, prompts, n_new, device):
    seqs = eng.generate(prompts, SamplingParams(max_tokens=n_new, temperature=0.0, ignore_eos=True))
    agree = total = 0
    for s in seqs:
        assert len(s.output_ids) == n_new
        for t in range(n_new):
            lg = _full_logits(eng.model, s.prompt_ids + s.output_ids[:t], device)
            top2 = torch.topk(lg, 2).values
            total += 1
            if int(lg.argmax()) == s.output_ids[t]:
                agree += 1
            else:  # only acceptable on a near-tie (bf16 rounding differs between the two paths)
                assert float(top2[0] - lg[s.output_ids[t]]) < 0.05 * float(top2[0].abs() + 1)
    assert agree / total > 0.9


@pytest.mark.parametrize("model", ["llama-tiny", "mixtral-tiny", "gpt2-tiny"])
def test_cpu_decode_matches_recompute(model):
    eng = LLMEngine(EngineConfig(model=model, max_num_seqs=4, max_model_len=256, num_blocks=64, use_graphs=False),
                    device="cpu")
    _check_greedy_consistency(eng, ["pod crashloop in kube-system", "node-003 NotReady 为什么", "x" * 40], 6, "cpu")


def test_scheduler_preempts_instead_of_failing():
    eng = LLMEngine(EngineConfig(model="llama-tiny", max_num_seqs=8, max_model_len=256, num_blocks=12,
                                 use_graphs=False), device="cpu")
    seqs = eng.generate(["a" * 30] * 6, SamplingParams(max_tokens=24, temperature=0.0, ignore_eos=True))
    assert all(len(s.output_ids) == 24 for s in seqs)
    assert eng.counters["preemptions"] > 0
    assert eng.blocks.num_free == 12


@pytest.mark.gpu
def test_gpu_decode_graphs_match_recompute():
    eng = LLMEngine(EngineConfig(model="llama-tiny-d128", max_num_seqs=8, max_model_len=1024, num_blocks=512),
                    device="cuda")
    eng.warmup()
    assert eng.runner.graphs
    long_prompt = "集群状态概览: " + "node-001 CPU=93.1% [资源压力]\n" * 40  # > 1 decode partition
    _check_greedy_consistency(eng, ["why is pod default/api not ready?", long_prompt, "x" * 300], 8, "cuda")


@pytest.mark.gpu
def test_gpu_graph_replay_equals_eager():
    cfg = dict(model="llama-tiny-d128", max_num_seqs=8, max_model_len=1024, num_blocks=512, seed=3)
    prompts = ["kube-system coredns CrashLoopBackOff", "MEM=95.9% [资源压力]" * 20]
    p = SamplingParams(max_tokens=12, temperature=0.0, ignore_eos=True)
    a = LLMEngine(EngineConfig(**cfg), device="cuda")
    a.warmup()
    b = LLMEngine(EngineConfig(**cfg, use_graphs=False), device="cuda")
    oa = [s.output_ids for s in a.generate(prompts, p)]
    ob = [s.output_ids for s in b.generate(prompts, p)]
    assert oa == ob


def test_prefix_caching_reuses_blocks_and_matches_uncached():
    """Prompts sharing a long prefix: the second wave maps the cached blocks (paged prefill of the
    suffix only) and generates exactly what an engine without prefix caching generates."""
    from k8s_llm_monitor_amd.engine import EngineConfig, LLMEngine, SamplingParams

    shared = "集群状态概览: node-000 NotReady, payments-api CrashLoopBackOff, " * 6
    prompts = [shared + f"问题 {i}: 为什么?" for i in range(3)]
    sp = SamplingParams(max_tokens=6, temperature=0.0, ignore_eos=True)
    outs = {}
    for pc in (True, False):
        eng = LLMEngine(EngineConfig(model="llama-tiny", max_num_seqs=4, max_model_len=512, num_blocks=128,
                                     use_graphs=False, seed=2, prefix_caching=pc, dtype="float32"), device="cpu")
        first = eng.generate(prompts[:1], sp)  # populates the cache
        rest = eng.generate(prompts[1:], sp)
        outs[pc] = [s.output_ids for s in first + rest]
        if pc:
            assert eng.blocks.stats()["prefix_cached_tokens"] >= 2 * 16
            assert all(s.num_cached == 0 for s in rest)  # released at finish
    assert outs[True] == outs[False]


def test_chunked_prefill_matches_whole_prompt_prefill():
    """A prefill budget far below the prompt lengths: every prompt is prefilled in chunks over
    several steps (later chunks attend the earlier ones from the paged cache); greedy outputs equal
    those of whole-prompt prefill, and no step computes more than the budget."""
    prompts = ["集群状态概览: node-000 NotReady, payments-api CrashLoopBackOff " * 3, "why is coredns failing? " * 4,
               "短"]
    sp = SamplingParams(max_tokens=5, temperature=0.0, ignore_eos=True)
    outs = {}
    for budget in (4096, 40):
        eng = LLMEngine(EngineConfig(model="llama-tiny", max_num_seqs=4, max_model_len=512, num_blocks=128,
                                     use_graphs=False, seed=5, dtype="float32", max_prefill_tokens=budget,
                                     prefix_caching=False), device="cpu")
        eng.trace = []
        seqs = eng.generate(prompts, sp)
        outs[budget] = [s.output_ids for s in seqs]
        chunks = [e[3] for e in eng.trace if e[1] == "prefill"]
        assert max(chunks) <= budget
        if budget == 40:
            assert len(chunks) >= sum(len(s.prompt_ids) for s in seqs) // 40
            assert eng.runner.n_steps["prefill_context_tokens"] > 0
    assert outs[4096] == outs[40]


def test_scheduler_chunks_and_defers_decode():
    from k8s_llm_monitor_amd.engine.block_manager import BlockManager
    from k8s_llm_monitor_amd.engine.scheduler import Scheduler, SchedulerConfig
    from k8s_llm_monitor_amd.engine.sequence import Sequence

    s = Scheduler(SchedulerConfig(max_num_seqs=4, max_prefill_tokens=32), BlockManager(64, use_native=False))
    a = Sequence(prompt_ids=list(range(70)), params=SamplingParams())
    b = Sequence(prompt_ids=list(range(10)), params=SamplingParams())
    s.add(a)
    s.add(b)
    p1 = s.schedule()
    assert p1.is_prefill and [q.chunk for q in p1.seqs] == [32]  # a's first chunk fills the budget
    assert not s.chunk_done(a)
    p2 = s.schedule()  # a's next chunk comes first and uses the whole budget
    assert p2.is_prefill and p2.seqs == [a] and a.chunk == 32
    s.chunk_done(a)
    p3 = s.schedule()
    assert p3.is_prefill and p3.seqs == [a, b] and (a.chunk, b.chunk) == (6, 10)
    assert s.chunk_done(a) and s.chunk_done(b)
    a.output_ids.append(1)
    b.output_ids.append(1)
    p4 = s.schedule()
    assert not p4.is_prefill and p4.seqs == [a, b]
    # without chunking a prompt larger than the budget still runs whole (alone)
    s2 = Scheduler(SchedulerConfig(max_num_seqs=4, max_prefill_tokens=32, chunked_prefill=False),
                   BlockManager(64, use_native=False))
    c = Sequence(prompt_ids=list(range(70)), params=SamplingParams())
    s2.add(c)
    assert s2.schedule().seqs[0].chunk == 70


@pytest.mark.gpu
def test_gpu_chunked_prefill_matches_whole():
    """Chunked prefill on the GPU path (paged flash prefill over earlier chunks, hipGraph decode)."""
    prompts = ["集群状态概览: " + "node-001 CPU=93.1% [资源压力]\n" * 30, "kube-system coredns CrashLoopBackOff " * 8]
    sp = SamplingParams(max_tokens=8, temperature=0.0, ignore_eos=True)
    outs = {}
    for budget in (16384, 100):
        eng = LLMEngine(EngineConfig(model="llama-tiny-d128", max_num_seqs=8, max_model_len=1024, num_blocks=512,
                                     seed=4, max_prefill_tokens=budget, prefix_caching=False), device="cuda")
        eng.warmup()
        outs[budget] = [s.output_ids for s in eng.generate(prompts, sp)]
        if budget == 100:
            assert eng.counters["prefill_steps"] >= 4
    assert outs[16384] == outs[100]


@pytest.mark.gpu
def test_gpu_moe_decode_grouped_skinny_matches_recompute():
    """Mixtral-shaped model on the GPU: grouped-skinny MoE decode in hipGraphs vs full recompute."""
    eng = LLMEngine(EngineConfig(model="mixtral-tiny-d128", max_num_seqs=8, max_model_len=1024, num_blocks=256),
                    device="cuda")
    eng.warmup()
    L0 = eng.model.layers[0]
    assert eng.runner.graphs and ("w13_pg" in L0 or "w13_dg" in L0)
    assert eng.model._packed and L0["w13"] is L0["w13_dg"]  # ONE_LAYOUT: the packed experts are the weights
    _check_greedy_consistency(eng, ["why is pod default/api not ready?", "kube-system coredns " * 20, "x" * 100],
                              8, "cuda")


def test_scheduler_admits_up_to_max_num_seqs_in_one_step():
    """Regression: sequences admitted in this step count once against max_num_seqs."""
    from k8s_llm_monitor_amd.engine.block_manager import BlockManager
    from k8s_llm_monitor_amd.engine.scheduler import Scheduler, SchedulerConfig
    from k8s_llm_monitor_amd.engine.sequence import Sequence

    s = Scheduler(SchedulerConfig(max_num_seqs=8, max_prefill_tokens=4096), BlockManager(256, use_native=False))
    for _ in range(10):
        s.add(Sequence(prompt_ids=list(range(20)), params=SamplingParams()))
    p = s.schedule()
    assert p.is_prefill and len(p.seqs) == 8 and len(s.running) == 8 and len(s.waiting) == 2


def test_service_coalesces_a_burst_into_one_prefill():
    """An idle engine receiving a burst (requests 1 ms apart) starts with one prefill of the
    burst, not a lone first prompt (admission coalescing window)."""
    import threading
    import time

    from k8s_llm_monitor_amd.engine import EngineService

    eng = LLMEngine(EngineConfig(model="llama-tiny", max_num_seqs=16, max_model_len=256, num_blocks=128,
                                 use_graphs=False, admit_gap_ms=50.0, admit_window_ms=400.0), device="cpu")
    eng.trace = []
    svc = EngineService(eng)
    futs = []

    def burst():
        for i in range(8):
            futs.append(svc.submit(f"pod-{i} OOMKilled", SamplingParams(max_tokens=2, ignore_eos=True)))
            time.sleep(0.001)

    t = threading.Thread(target=burst)
    t.start()
    t.join()
    for f in futs:
        f.result(timeout=60)
    svc.close()
    first = next(e for e in eng.trace if e[1] == "prefill")
    assert first[2] == 8


def test_service_coalescing_stops_at_a_full_prefill_budget():
    """Admission coalescing ends as soon as the queued prompts fill one prefill step
    (max_prefill_tokens): the first prefill does not wait out the window for the rest of a burst."""
    import time

    from k8s_llm_monitor_amd.engine import EngineService

    eng = LLMEngine(EngineConfig(model="llama-tiny", max_num_seqs=16, max_model_len=256, num_blocks=256,
                                 use_graphs=False, max_prefill_tokens=64, admit_gap_ms=400.0,
                                 admit_window_ms=2000.0), device="cpu")
    eng.trace = []
    svc = EngineService(eng)
    prompt = "pod default/api-gateway CrashLoopBackOff restarted 12 times " * 3  # > 64 tokens alone
    t0 = time.perf_counter()
    fut = svc.submit(prompt, SamplingParams(max_tokens=1, ignore_eos=True))
    fut.result(timeout=60)
    dt = time.perf_counter() - t0
    svc.close()
    assert dt < 0.4, f"first prefill waited {dt:.3f} s for more arrivals with a full budget queued"


def test_decode_staging_layout_and_resolve_ids_cpu():
    """The packed decode-input buffer: field views are disjoint, in the documented order, float
    fields bit-cast, and the copied prefix covers the per-row fields plus the live block-table rows;
    resolve_ids' CPU path picks the previous step's token where src >= 0."""
    import numpy as np
    import torch

    from k8s_llm_monitor_amd import ops
    from k8s_llm_monitor_amd.engine.runner import _Staging

    B, mb = 8, 5
    st = _Staging(B, mb, pin=False)
    assert st.h_all.numel() == _Staging.size(B, mb) == 8 * B + B * mb
    st.n_ids[:] = 1
    st.n_src[:] = 2
    st.n_pos[:] = 3
    st.n_slots[:] = 4
    st.n_lens[:] = 5
    st.n_topk[:] = 6
    st.n_temp[:] = 0.5
    st.n_topp[:] = 0.25
    st.n_bt[:] = 9
    raw = st.h_all.numpy()
    for i, v in enumerate([1, 2, 3, 4, 5, 6]):
        assert (raw[i * B:(i + 1) * B] == v).all()
    assert (raw[6 * B:7 * B].view(np.float32) == 0.5).all() and (raw[7 * B:8 * B].view(np.float32) == 0.25).all()
    assert (raw[8 * B:] == 9).all()
    assert _Staging.prefix(B, mb, 3) == 8 * B + 3 * mb
    dev = torch.zeros(_Staging.size(B, mb), dtype=torch.int32)
    views = _Staging.views(dev, B, mb)
    assert views[6].dtype == torch.float32 and views[8].shape == (B, mb)
    ids = torch.tensor([10, 11, 12, 13], dtype=torch.int32)
    src = torch.tensor([-1, 2, -1, 0], dtype=torch.int32)
    prev = torch.tensor([100, 101, 102, 103], dtype=torch.int32)
    assert ops.resolve_ids(ids, src, prev).tolist() == [10, 102, 12, 100]


def test_pipelined_prefill_matches_sync_engine():
    """Prefill-only steps are enqueued before the previous one is read back (pending_first): a
    burst prefilled over several pipelined steps (chunked prompts, a mid-burst abort) yields the
    same greedy tokens as the synchronous engine, and no KV block leaks."""
    prompts = [f"pod-{i} CrashLoopBackOff on node-{i:03d}, restarts={i * 7}; " * (3 + i % 3) for i in range(6)]
    sp = SamplingParams(max_tokens=5, temperature=0.0, ignore_eos=True)
    outs = {}
    for pipe in (True, False):
        eng = LLMEngine(EngineConfig(model="llama-tiny", max_num_seqs=8, max_model_len=512, num_blocks=256,
                                     use_graphs=False, seed=3, dtype="float32", prefix_caching=False,
                                     max_prefill_tokens=48, pipeline=pipe), device="cpu")
        seqs = [eng.add_request(p, sp) for p in prompts]
        extra = eng.add_request("aborted while its prefill is in flight " * 4, sp)
        eng.step()
        eng.step()
        eng.abort(extra)
        while eng.has_work():
            eng.step()
        assert all(s.status == SeqStatus.FINISHED and len(s.output_ids) == 5 for s in seqs)
        assert eng.blocks.num_free == 256
        outs[pipe] = [s.output_ids for s in seqs]
    assert outs[True] == outs[False]


def test_attention_row_order_pairs_long_and_short():
    """64-row decode graph: rows 0..31 are the 32 longest contexts (longest first), rows 32..63
    the rest shortest first, so rows z and z + 32 (one CU in the paged-attention grid) pair the
    k-th longest with the k-th shortest; other bucket sizes are longest first."""
    import random
    import types

    from k8s_llm_monitor_amd.engine.engine import LLMEngine

    rng = random.Random(0)
    seqs = [types.SimpleNamespace(num_tokens=rng.randint(1200, 2400), seq_id=i) for i in range(64)]
    eng = types.SimpleNamespace(runner=types.SimpleNamespace(graphs={64: object()}, bucket_for=lambda n: 64))
    out = LLMEngine._attention_row_order(eng, list(seqs))
    assert sorted(q.seq_id for q in out) == list(range(64))
    lens = [q.num_tokens for q in out]
    srt = sorted(lens, reverse=True)
    assert lens[:32] == srt[:32] and lens[32:] == srt[32:][::-1]
    for z in range(32):  # the pair on one CU: k-th longest with k-th shortest
        assert lens[z] == srt[z] and lens[z + 32] == srt[63 - z]
    eng.runner.bucket_for = lambda n: 32
    out = LLMEngine._attention_row_order(eng, list(seqs[:20]))
    assert [q.num_tokens for q in out] == sorted((q.num_tokens for q in seqs[:20]), reverse=True)
