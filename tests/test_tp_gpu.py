"""Tensor-parallel decode on the GPU (VERDICT r1 'do this' #2): two TP ranks as two processes
sharing the box's one MI355X run the FULL engine - prefill, mixed prefill+decode steps and
pipelined hipGraph decode with the collectives captured in the graph (the one-shot IPC all-reduce /
all-gather: RCCL refuses two ranks on one device, so the process group is gloo and nothing in the
decode graph may be a gloo call) - with the leader handing steps to the worker over the
shared-memory step bus.  Every generated token must be the TP=1 model's greedy choice on a full
recompute (or a bf16 near-tie), and no collective may have timed out."""
import os
import socket

import pytest
import torch


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


PROMPTS = ["why is pod default/api not ready?", "集群状态概览: " + "node-001 CPU=93.1% [资源压力]\n" * 12]
LATE = "kube-system coredns CrashLoopBackOff " * 6


def _rank(rank: int, world: int, port: int, q) -> None:
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    os.environ.pop("K8SLLM_CUSTOM_AR", None)  # default: on at TP > 1
    from k8s_llm_monitor_amd.engine import EngineConfig, LLMEngine, SamplingParams
    from k8s_llm_monitor_amd.parallel.state import destroy, init_parallel

    try:
        ps = init_parallel(tp_size=world, device="cuda:0", backend="gloo")
        assert ps.custom_ar is not None
        eng = LLMEngine(EngineConfig(model="llama-tiny-d128", max_num_seqs=8, max_model_len=1024, num_blocks=256,
                                     seed=9, tp_size=world, max_prefill_tokens=96, mixed_prefill_tokens=64),
                        device="cuda:0", pstate=ps)
        eng.warmup()
        assert eng.runner.graphs, "decode graphs were not captured"
        out = None
        if ps.tp_rank == 0:
            sp = SamplingParams(max_tokens=10, temperature=0.0, ignore_eos=True)
            seqs = [eng.add_request(p, sp) for p in PROMPTS]
            for _ in range(4):
                eng.step()
            seqs.append(eng.add_request(LATE, sp))
            while eng.has_work():
                eng.step()
            out = {"tokens": [(s.prompt_ids, s.output_ids) for s in seqs], "mixed": eng.counters["mixed_steps"],
                   "decode": eng.counters["decode_steps"], "bus": type(eng.bus).__name__}
            eng.stop_workers()
        else:
            eng.worker_loop()
        torch.cuda.synchronize()
        err = ps.custom_ar.error()
        eng.bus.close()
        ps.custom_ar.close()
        destroy()
        q.put((rank, out, err))
    except BaseException as e:  # noqa: BLE001
        import traceback

        q.put((rank, repr(e) + traceback.format_exc(), True))


def _full_logits(model, ids):
    from k8s_llm_monitor_amd.models import AttnMeta

    n = len(ids)
    t = torch.tensor(ids, dtype=torch.int32, device="cuda")
    meta = AttnMeta(is_prefill=True, positions=torch.arange(n, dtype=torch.int32, device="cuda"),
                    slot_mapping=torch.full((n,), -1, dtype=torch.int32, device="cuda"),
                    cu_seqlens=torch.tensor([0, n], dtype=torch.int32, device="cuda"),
                    logits_idx=torch.tensor([n - 1], device="cuda"))
    return model.forward(t, meta, None)[0].float()


@pytest.mark.gpu
def test_gpu_tp2_engine_graph_decode_matches_tp1_model():
    import multiprocessing as mp

    from k8s_llm_monitor_amd.models import CausalLM, get_config
    from k8s_llm_monitor_amd.parallel.state import ParallelState

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank, args=(r, 2, port, q), daemon=True) for r in range(2)]
    for p in procs:
        p.start()
    res = {}
    try:
        for _ in procs:
            rank, out, err = q.get(timeout=240)
            res[rank] = (out, err)
    finally:
        for p in procs:
            p.join(timeout=30)
            if p.is_alive():
                p.terminate()
    for rank, (out, err) in res.items():
        assert not isinstance(out, str), out
        assert err is False, f"rank {rank}: custom all-reduce timed out"
    out = res[0][0]
    assert out["bus"] == "ShmStepBus" and out["mixed"] > 0 and out["decode"] > 0
    ref = CausalLM(get_config("llama-tiny-d128"), device="cuda", seed=9,
                   pstate=ParallelState(device=torch.device("cuda", 0)))
    agree = total = 0
    for prompt, toks in out["tokens"]:
        assert len(toks) == 10
        for t in range(len(toks)):
            lg = _full_logits(ref, prompt + toks[:t])
            total += 1
            if int(lg.argmax()) == toks[t]:
                agree += 1
            else:  # only on a bf16 near-tie (TP sums its row-parallel partials in another order)
                top = float(lg.max())
                assert top - float(lg[toks[t]]) < 0.05 * (abs(top) + 1), (t, top, float(lg[toks[t]]))
    assert agree / total > 0.9


def _rank8b(rank: int, world: int, port: int, q) -> None:
    """TP=2 rank at Llama-3-8B dimensions (2 layers): hipGraph decode with the fused row-parallel
    tails (custom_ar.hip car_fused_tail_kernel) and the one-shot logits gather."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    os.environ.pop("K8SLLM_CUSTOM_AR", None)
    from k8s_llm_monitor_amd.engine import EngineConfig, LLMEngine, SamplingParams
    from k8s_llm_monitor_amd.parallel.state import destroy, init_parallel

    try:
        ps = init_parallel(tp_size=world, device="cuda:0", backend="gloo")
        assert ps.custom_ar is not None
        eng = LLMEngine(EngineConfig(model="llama-3-8b", model_overrides={"n_layers": 2}, max_num_seqs=8,
                                     max_model_len=1024, kv_cache_gb=0.5, seed=21, tp_size=world),
                        device="cuda:0", pstate=ps)
        eng.warmup()
        out = None
        if ps.tp_rank == 0:
            sp = SamplingParams(max_tokens=12, temperature=0.0, ignore_eos=True)
            seqs = eng.generate(PROMPTS + [LATE], sp)
            out = {"tokens": [(s.prompt_ids, s.output_ids) for s in seqs], "decode": eng.counters["decode_steps"]}
            eng.stop_workers()
        else:
            eng.worker_loop()
        torch.cuda.synchronize()
        err = ps.custom_ar.error()
        eng.bus.close()
        ps.custom_ar.close()
        destroy()
        q.put((rank, out, err))
    except BaseException as e:  # noqa: BLE001
        import traceback

        q.put((rank, repr(e) + traceback.format_exc(), True))


@pytest.mark.gpu
def test_gpu_tp2_llama8b_dims_matches_fp32_reference():
    """VERDICT r2 'do this' #3: TP=2 at Llama-3-8B dimensions (d 4096, 32/8 heads, ff 14336, vocab
    128256; 2 layers) through the engine's graph decode, every greedy token checked against an fp32
    CPU reference holding the same weights (the TP=1 GPU model with the same seed, copied to fp32:
    TP shards are slices of exactly those tensors) - the reference argmax or a bf16 near-tie."""
    import multiprocessing as mp

    from k8s_llm_monitor_amd.engine import EngineConfig, LLMEngine
    from test_real_shape_gpu import _fp32_reference, _logits

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank8b, args=(r, 2, port, q), daemon=True) for r in range(2)]
    for p in procs:
        p.start()
    res = {}
    try:
        for _ in procs:
            rank, out, err = q.get(timeout=300)
            res[rank] = (out, err)
    finally:
        for p in procs:
            p.join(timeout=30)
            if p.is_alive():
                p.terminate()
    for rank, (out, err) in res.items():
        assert not isinstance(out, str), out
        assert err is False, f"rank {rank}: custom all-reduce timed out"
    out = res[0][0]
    assert out["decode"] > 0
    torch.set_num_threads(16)
    eng1 = LLMEngine(EngineConfig(model="llama-3-8b", model_overrides={"n_layers": 2}, max_num_seqs=8,
                                  max_model_len=1024, kv_cache_gb=0.25, seed=21, use_graphs=False), device="cuda")
    ref = _fp32_reference(eng1.model)
    del eng1
    torch.cuda.empty_cache()
    agree = total = 0
    for prompt, toks in out["tokens"]:
        assert len(toks) == 12
        ids = prompt + toks
        p = len(prompt)
        lr = _logits(ref, ids, list(range(p - 1, p - 1 + len(toks))), "cpu")
        scale = float(lr.abs().max())
        for t, tok in enumerate(toks):
            total += 1
            if int(lr[t].argmax()) == tok:
                agree += 1
            else:  # a bf16 near-tie only
                top = float(lr[t].max())
                assert top - float(lr[t][tok]) < 0.02 * scale, (t, top, float(lr[t][tok]), scale)
    assert agree / total >= 0.9, (agree, total)


def _rank_ep(rank: int, world: int, port: int, q) -> None:
    """TP/EP=2 Mixtral-shaped MoE layer at decode: the expert-parallel all-to-all form (IPC
    all-to-all + grouped skinny expert kernels), eager and replayed from a hipGraph, against the
    replicated form (every rank runs its experts on every row, then one all-reduce)."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    os.environ.pop("K8SLLM_CUSTOM_AR", None)
    from k8s_llm_monitor_amd.models import AttnMeta, CausalLM, get_config
    from k8s_llm_monitor_amd.parallel.comm import tp_all_reduce
    from k8s_llm_monitor_amd.parallel.state import destroy, init_parallel

    try:
        ps = init_parallel(tp_size=world, device="cuda:0", backend="gloo")
        cfg = get_config("mixtral-tiny").replace(d_model=512, ffn_dim=1024)
        model = CausalLM(cfg, device="cuda", seed=13, pstate=ps)
        L = model.layers[0]
        res = []
        for M in (1, 24, 64):
            g = torch.Generator(device="cuda").manual_seed(100 + M)
            x = (torch.randn(M, cfg.d_model, device="cuda", generator=g) * 0.5).to(torch.bfloat16)
            meta = AttnMeta(is_prefill=False, positions=torch.zeros(M, dtype=torch.int32, device="cuda"),
                            slot_mapping=torch.full((M,), -1, dtype=torch.int32, device="cuda"))
            y_ref = tp_all_reduce(model._moe(L, x, meta), ps).float()
            y = model._moe_a2a_decode(L, x).float()
            # the same layer captured and replayed (the decode step is a hipGraph)
            xs = x.clone()
            s = torch.cuda.Stream()
            s.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(s):
                model._moe_a2a_decode(L, xs)
            torch.cuda.current_stream().wait_stream(s)
            gr = torch.cuda.CUDAGraph()
            with torch.cuda.graph(gr):
                yg = model._moe_a2a_decode(L, xs)
            gr.replay()
            torch.cuda.synchronize()
            scale = float(y_ref.abs().max()) + 1e-6
            res.append((M, float((y - y_ref).abs().max()) / scale, float((yg.float() - y).abs().max()) / scale))
        err = ps.custom_ar.error()
        n_a2a = ps.custom_ar.n_a2a_launches
        ps.custom_ar.close()
        destroy()
        q.put((rank, res, err, n_a2a))
    except BaseException as e:  # noqa: BLE001
        import traceback

        q.put((rank, repr(e) + traceback.format_exc(), True, 0))


@pytest.mark.gpu
def test_gpu_ep2_a2a_decode_matches_replicated():
    """VERDICT r2 'do this' #4: the EP all-to-all MoE decode on the hand-written path (IPC
    all-to-all kernel + grouped skinny expert GEMMs) equals the replicated form within bf16
    rounding, eagerly and replayed from a captured hipGraph, on two TP ranks sharing the GPU."""
    import multiprocessing as mp

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank_ep, args=(r, 2, port, q), daemon=True) for r in range(2)]
    for p in procs:
        p.start()
    out = {}
    try:
        for _ in procs:
            rank, res, err, n_a2a = q.get(timeout=300)
            out[rank] = (res, err, n_a2a)
    finally:
        for p in procs:
            p.join(timeout=30)
            if p.is_alive():
                p.terminate()
    for rank, (res, err, n_a2a) in out.items():
        assert not isinstance(res, str), res
        assert err is False, f"rank {rank}: a collective timed out"
        assert n_a2a > 0, "the IPC all-to-all kernel was never launched"
        for M, rel, rel_graph in res:
            assert rel < 2e-2, (rank, M, rel)
            assert rel_graph == 0.0, (rank, M, rel_graph)


def _overlap_rank(rank: int, world: int, port: int, q) -> None:
    """TP prefill as two overlapped micro-batches (the IPC all-reduces on the comm stream) against
    the serial form on the same ranks: 4 sequences of Llama-3-8B-shaped layers (d 4096, 2 layers)
    so the micro-batches' all-reduces fit the IPC staging buffer.  Both micro-batches keep >= 1024
    rows, so every projection stays on the tile GEMM, whose per-row results do not depend on the
    row count (a micro-batch under TILE_MIN_M would switch to hipBLASLt: right, not bit-equal)."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    os.environ.pop("K8SLLM_CUSTOM_AR", None)
    import numpy as np

    from k8s_llm_monitor_amd import ops
    from k8s_llm_monitor_amd.engine.runner import ModelRunner
    from k8s_llm_monitor_amd.models import AttnMeta, CausalLM, get_config
    from k8s_llm_monitor_amd.parallel.state import destroy, init_parallel

    try:
        ps = init_parallel(tp_size=world, device="cuda:0", backend="gloo")
        assert ps.custom_ar is not None
        dev = ps.device
        cfg = get_config("llama-3-8b").replace(n_layers=2)
        m = CausalLM(cfg, device=dev, seed=4, pstate=ps)
        lens = [1100, 300, 800, 400]  # micro-batches of 1400 / 1200 rows: both on the tile GEMM
        cu = np.concatenate([[0], np.cumsum(lens)]).astype(np.int32)
        T = int(cu[-1])
        ids = (torch.arange(T, dtype=torch.int32, device=dev) * 7919) % cfg.vocab_size
        pos = torch.cat([torch.arange(n, dtype=torch.int32) for n in lens]).to(dev)

        def meta_for(c, p):
            qs, st = ops.prefill_qblocks([int(v) for v in c])
            return AttnMeta(is_prefill=True, positions=p,
                            slot_mapping=torch.full((len(p),), -1, dtype=torch.int32, device=dev),
                            cu_seqlens=torch.tensor(c, dtype=torch.int32, device=dev),
                            qb_seq=torch.tensor(qs, dtype=torch.int32, device=dev),
                            qb_start=torch.tensor(st, dtype=torch.int32, device=dev),
                            logits_idx=torch.tensor(np.asarray(c[1:]) - 1, dtype=torch.int64, device=dev))

        kA = ModelRunner._micro_split(cu, 0, min_rows=0)
        TA = int(cu[kA])
        full = meta_for(cu, pos)
        full.micro = (meta_for(cu[: kA + 1], pos[:TA]), meta_for(cu[kA:] - cu[kA], pos[TA:]), TA)
        with torch.no_grad():
            serial = m.forward(ids, meta_for(cu, pos), None)
            outs = [m.forward(ids, full, None) for _ in range(3)]  # back to back: comm-stream reuse
        torch.cuda.synchronize()
        same = all(torch.equal(o, serial) for o in outs)
        diff = max(float((o.float() - serial.float()).abs().max()) for o in outs)
        err = ps.custom_ar.error()
        ps.custom_ar.close()
        destroy()
        q.put((rank, (kA, same, diff), err))
    except BaseException as e:  # noqa: BLE001
        import traceback

        q.put((rank, repr(e) + traceback.format_exc(), True))


@pytest.mark.gpu
def test_gpu_tp2_prefill_overlap_matches_serial():
    """VERDICT r4 item 3 on the GPU: the overlapped micro-batch prefill (async IPC all-reduces on
    the comm stream, compute on the current stream) is bit-identical to the serial TP prefill, and
    no all-reduce timed out (the 64-workgroup cap keeps a spinning all-reduce from locking the
    peer's GEMMs off the shared GPU)."""
    import multiprocessing as mp

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_overlap_rank, args=(r, 2, port, q), daemon=True) for r in range(2)]
    for p in procs:
        p.start()
    res = {}
    try:
        for _ in procs:
            rank, out, err = q.get(timeout=240)
            res[rank] = (out, err)
    finally:
        for p in procs:
            p.join(timeout=30)
            if p.is_alive():
                p.terminate()
    for rank, (out, err) in res.items():
        assert not isinstance(out, str), out
        assert err is False, f"rank {rank}: custom all-reduce timed out"
        kA, same, diff = out
        assert kA == 2 and same, f"rank {rank}: overlapped prefill differs from serial by {diff}"
