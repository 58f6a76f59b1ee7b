"""Real-shape GPU parity (VERDICT r1 'do this' #9): the full engine path - paged prefill, the skinny
MFMA decode GEMMs over fragment-packed weights inside hipGraphs, HIP attention / RoPE / norms and
the sampler - at Llama-3-8B dimensions (d 4096, 32/8 heads, ff 14336, vocab 128256, theta 5e5; two
layers) and at Llama-3-70B dimensions (d 8192, 64/8 heads, ff 28672; one layer), against an fp32
CPU reference model holding the SAME weights (copied from the GPU model).

Checks: (1) prefill logits of the bf16 GPU forward vs the fp32 reference: max-abs error bounded
relative to the logit scale; (2) 16 greedy decode steps through the engine: every generated token
is the fp32 reference's argmax on the teacher-forced sequence, or a provable near-tie (its logit
within twice the measured bf16 logit error of the max)."""
import pytest
import torch


def _fp32_reference(gpu_model):
    from k8s_llm_monitor_amd.models import CausalLM
    from k8s_llm_monitor_amd.parallel.state import ParallelState

    CausalLM.SKINNY_DECODE = False  # the reference runs the plain row-major path only
    try:
        ref = CausalLM(gpu_model.cfg, device="cpu", dtype=torch.float32, pstate=ParallelState(), init="empty")
    finally:
        CausalLM.SKINNY_DECODE = True
    ref.copy_weights_from(gpu_model)
    return ref


def _logits(model, ids, rows, device):
    from k8s_llm_monitor_amd.models import AttnMeta

    n = len(ids)
    t = torch.tensor(ids, dtype=torch.int32, device=device)
    meta = AttnMeta(is_prefill=True, positions=torch.arange(n, dtype=torch.int32, device=device),
                    slot_mapping=torch.full((n,), -1, dtype=torch.int32, device=device),
                    cu_seqlens=torch.tensor([0, n], dtype=torch.int32, device=device),
                    logits_idx=torch.tensor(rows, device=device))
    return model.forward(t, meta, None).float().cpu()


@pytest.mark.gpu
@pytest.mark.parametrize("model,layers", [("llama-3-8b", 2), ("llama-3-70b", 1), ("mixtral-8x7b", 1)])
def test_gpu_real_shape_engine_matches_fp32_reference(model, layers):
    """Mixtral-8x7B dimensions (d 4096, 8 experts of ff 14336, top-2) exercise the grouped skinny
    MoE decode kernels inside the decode hipGraph (VERDICT r2 'do this' #7)."""
    from k8s_llm_monitor_amd.engine import EngineConfig, LLMEngine, SamplingParams

    torch.set_num_threads(16)
    eng = LLMEngine(EngineConfig(model=model, model_overrides={"n_layers": layers}, max_num_seqs=8,
                                 max_model_len=2048, kv_cache_gb=1.0, seed=21), device="cuda")
    eng.warmup()
    L0 = eng.model.layers[0]
    assert eng.runner.graphs and ("wqkv_p" in L0 or "wqkv_d" in L0), "skinny decode path not active"
    if model == "llama-3-8b":  # dense Llama: one resident copy, packed (CausalLM.ONE_LAYOUT)
        assert eng.model._packed and L0["w13"] is L0["w13_d"] and "w13_p" not in L0
    prompts = ["集群状态概览: node-001 CPU=93.1% [资源压力] MEM=88% 为什么我的pod频繁重启？ " * 3,
               "Why is pod default/api-gateway not ready? kube-system coredns CrashLoopBackOff " * 2,
               "node-007 NotReady, payments-api OOMKilled x12"]
    n_new = 16
    seqs = eng.generate(prompts, SamplingParams(max_tokens=n_new, temperature=0.0, ignore_eos=True))
    ref = _fp32_reference(eng.model)
    for s in seqs:
        assert len(s.output_ids) == n_new
        ids = s.prompt_ids + s.output_ids
        p = len(s.prompt_ids)
        rows = list(range(p - 1, p - 1 + n_new))
        lr = _logits(ref, ids, rows, "cpu")  # [16, V] fp32 reference, teacher-forced
        lg = _logits(eng.model, ids, rows, "cuda")  # the bf16 GPU prefill path on the same rows
        scale = float(lr.abs().max())
        err = float((lg - lr).abs().max())
        assert err < 0.03 * scale, f"{model}: prefill logits max-abs err {err:.4f} vs scale {scale:.3f}"
        for t in range(n_new):
            top = float(lr[t].max())
            got = float(lr[t, s.output_ids[t]])
            assert top - got <= 2 * err + 1e-6, (
                f"{model} step {t}: token {s.output_ids[t]} logit {got:.4f} vs max {top:.4f} (bf16 err {err:.4f})")
    del eng
    torch.cuda.empty_cache()


@pytest.mark.gpu
@pytest.mark.parametrize("batch", [40, 64])
def test_gpu_real_shape_decode_batch64_matches_fp32_reference(batch):
    """The headline's decode batch: 64 rows through the skinny decode graph (M = 64 buckets, the
    deferred RMSNorm) at Llama-3-8B dimensions, against the fp32 CPU reference holding the same
    weights.  Every greedy token must be the reference's argmax on the teacher-forced sequence or a
    provable near-tie (within twice the measured bf16-vs-fp32 logit error of that sequence's GPU
    prefill forward).  Rows 33-64 exercise what batches of <= 32 never reach; 40 rows run the
    64-row graph with 24 padding rows."""
    from k8s_llm_monitor_amd.engine import EngineConfig, LLMEngine, SamplingParams

    torch.set_num_threads(16)
    eng = LLMEngine(EngineConfig(model="llama-3-8b", model_overrides={"n_layers": 2}, max_num_seqs=64,
                                 max_model_len=1024, kv_cache_gb=2.0, seed=5), device="cuda")
    eng.warmup()
    prompts = [f"node-{i:03d} CPU={30 + i}% pod payments-{i} restarts={i % 7} 为什么我的pod频繁重启？" for i in range(batch)]
    n_new = 8
    seqs = eng.generate(prompts, SamplingParams(max_tokens=n_new, temperature=0.0, ignore_eos=True))
    assert 64 in eng.stats()["graph_buckets"]
    ref = _fp32_reference(eng.model)
    for i, s in enumerate(seqs):
        ids = s.prompt_ids + s.output_ids
        p = len(s.prompt_ids)
        rows = list(range(p - 1, p - 1 + n_new))
        lr = _logits(ref, ids, rows, "cpu")
        lg = _logits(eng.model, ids, rows, "cuda")
        scale = float(lr.abs().max())
        err = float((lg - lr).abs().max())
        assert err < 0.03 * scale, f"row {i}: prefill logits max-abs err {err:.4f} vs scale {scale:.3f}"
        for t in range(n_new):
            top, got = float(lr[t].max()), float(lr[t, s.output_ids[t]])
            assert top - got <= 2 * err + 1e-6, (
                f"row {i} step {t}: token {s.output_ids[t]} logit {got:.4f} vs max {top:.4f} (bf16 err {err:.4f})")
    del eng
    torch.cuda.empty_cache()
