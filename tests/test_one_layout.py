"""ONE_LAYOUT: a dense Llama keeps ONE resident copy of every projection - the
decode GEMMs' fragment-packed layout, read by the prefill tile GEMM as well.  CPU forms: the
packed model computes what the row-major model computes (prefill and decode), its canonical
weights round-trip bit-exactly, and checkpoint export sees row-major tensors.  (GPU numerics of
the packed tile GEMM: test_gemm_tile_gpu.py; end to end: test_tile_real_shapes_gpu.py.)"""
import pytest
import torch

from k8s_llm_monitor_amd import ops
from k8s_llm_monitor_amd.models import AttnMeta, CausalLM, get_config


def _pair(monkeypatch, model="llama-tiny-d128"):
    cfg = get_config(model)
    monkeypatch.setattr(CausalLM, "ONE_LAYOUT", False)
    ref = CausalLM(cfg, device="cpu", dtype=torch.float32, seed=11)
    monkeypatch.setattr(CausalLM, "ONE_LAYOUT", "force")
    one = CausalLM(cfg, device="cpu", dtype=torch.float32, seed=11)
    return ref, one


@pytest.mark.parametrize("model", ["llama-tiny-d128", "mixtral-tiny-d128"])
def test_one_layout_single_packed_copy(monkeypatch, model):
    ref, one = _pair(monkeypatch, model)
    assert one._packed and not ref._packed and one._swg == 8
    for L, L0 in zip(one.layers, ref.layers):
        for key in ("wqkv", "wo", "w13", "w2"):
            moe = one.cfg.is_moe and key in ("w13", "w2")
            dk = key + ("_dg" if moe else "_d")
            assert L[key].dim() == (5 if moe else 4) and L[key] is L[dk]  # the decode copy IS the weight
            assert key + "_p" not in L and key + "_pg" not in L
            assert torch.equal(one.canonical(L, key), ref.canonical(L0, key))
    assert one.num_local_params() == ref.num_local_params()
    assert one.lm_head is one.lm_head_d and torch.equal(one.canonical_head(), ref.lm_head)
    x = torch.randn(70, ref.cfg.d_model)  # > 64 rows: the packed head in 64-row chunks
    assert (one._logits(x) - ref._logits(x)).abs().max().item() < 1e-4


@pytest.mark.parametrize("model", ["llama-tiny-d128", "mixtral-tiny-d128"])
def test_one_layout_prefill_and_decode_match_rowmajor(monkeypatch, model):
    ref, one = _pair(monkeypatch, model)
    bs, nb = 16, 8
    g = torch.Generator().manual_seed(0)
    kv0 = [(torch.randn(nb, ref.hkv, ref.D // 8, bs, 8, generator=g), torch.randn(nb, ref.hkv, ref.D, bs, generator=g))
           for _ in ref.layers]
    kv1 = [(k.clone(), v.clone()) for k, v in kv0]
    # prefill: two prompts of 5 and 9 tokens into blocks 0 and 1..2
    T = torch.tensor([5, 9])
    ids = torch.randint(0, 1000, (14,), generator=g, dtype=torch.int32)
    pos = torch.cat([torch.arange(5), torch.arange(9)]).to(torch.int32)
    slots = torch.cat([torch.arange(5), 16 + torch.arange(9)]).to(torch.int32)
    cu = torch.tensor([0, 5, 14], dtype=torch.int32)
    meta = AttnMeta(is_prefill=True, positions=pos, slot_mapping=slots, cu_seqlens=cu,
                    logits_idx=torch.tensor([4, 13]))
    a = ref.forward(ids, meta, kv0)
    b = one.forward(ids, meta, kv1)
    assert (a - b).abs().max().item() < 1e-4
    for (k0, v0), (k1, v1) in zip(kv0, kv1):
        assert (k0 - k1).abs().max().item() < 1e-5 and (v0 - v1).abs().max().item() < 1e-5
    # one decode step of both sequences
    lens = T + 1
    dm = AttnMeta(is_prefill=False, positions=(lens - 1).to(torch.int32), slot_mapping=torch.tensor([5, 25], dtype=torch.int32),
                  block_tables=torch.tensor([[0, 3], [1, 2]], dtype=torch.int32), seq_lens=lens.to(torch.int32))
    nid = torch.tensor([7, 99], dtype=torch.int32)
    a = ref.forward(nid, dm, kv0)
    b = one.forward(nid, dm, kv1)
    assert (a - b).abs().max().item() < 1e-4


@pytest.mark.parametrize("model", ["llama-tiny-d128", "mixtral-tiny-d128"])
def test_one_layout_checkpoint_export_is_rowmajor(monkeypatch, model):
    from k8s_llm_monitor_amd.models.checkpoint import hf_state_dict

    ref, one = _pair(monkeypatch, model)
    sd0 = dict(hf_state_dict(ref))
    sd1 = dict(hf_state_dict(one))
    assert sd0.keys() == sd1.keys()
    for k in sd0:
        assert torch.equal(sd0[k], sd1[k]), k


@pytest.mark.parametrize("model", ["llama-tiny-d128", "mixtral-tiny-d128"])
def test_one_layout_reinit_restores_rowmajor(monkeypatch, model):
    """_init_skinny over packed weights (e.g. after a DECODE_GEMM change) starts from the canonical
    tensors again instead of packing the packed copy."""
    ref, one = _pair(monkeypatch, model)
    monkeypatch.setattr(CausalLM, "ONE_LAYOUT", False)
    one._init_skinny()
    assert not one._packed
    for L, L0 in zip(one.layers, ref.layers):
        for key in ("wqkv", "wo", "w13", "w2"):
            assert L[key].dim() == L0[key].dim() and torch.equal(L[key], L0[key])


@pytest.mark.gpu
def test_one_layout_gpu_matches_two_layouts():
    """On the GPU the one packed copy gives the row-major model's logits: prefill (1300 tokens: the
    tile GEMMs with the fused norms, packed W and the per-16 SwiGLU pairing) and a decode step
    (the decode GEMMs read the same packed tensors either way)."""
    cfg = get_config("llama-tiny-d128")
    CausalLM.ONE_LAYOUT = False
    try:
        two = CausalLM(cfg, device="cuda", dtype=torch.bfloat16, seed=5)
    finally:
        CausalLM.ONE_LAYOUT = True
    one = CausalLM(cfg, device="cuda", dtype=torch.bfloat16, seed=5)
    assert one._packed and not two._packed
    n = 1300
    g = torch.Generator().manual_seed(1)
    ids = torch.randint(3, cfg.vocab_size, (n,), generator=g, dtype=torch.int32).cuda()
    rows = [0, 511, 1024, n - 1]
    meta = AttnMeta(is_prefill=True, positions=torch.arange(n, dtype=torch.int32, device="cuda"),
                    slot_mapping=torch.full((n,), -1, dtype=torch.int32, device="cuda"),
                    cu_seqlens=torch.tensor([0, n], dtype=torch.int32, device="cuda"),
                    logits_idx=torch.tensor(rows, device="cuda"))
    a = two.forward(ids, meta, None).float()
    b = one.forward(ids, meta, None).float()
    scale = float(a.abs().max())
    err = float((a - b).abs().max())
    assert err <= 1e-3 * scale, f"one layout vs two: max err {err} (scale {scale})"


def test_copy_weights_between_layouts(monkeypatch):
    """copy_weights_from moves weights between a packed (ONE_LAYOUT) and a row-major model in either
    direction (the GPU tests build their fp32 CPU references this way)."""
    ref, one = _pair(monkeypatch)
    cfg = get_config("llama-tiny-d128")
    monkeypatch.setattr(CausalLM, "ONE_LAYOUT", False)
    a = CausalLM(cfg, device="cpu", dtype=torch.float32, seed=99, init="empty")
    a.copy_weights_from(one)
    monkeypatch.setattr(CausalLM, "ONE_LAYOUT", "force")
    b = CausalLM(cfg, device="cpu", dtype=torch.float32, seed=99, init="empty")
    b.copy_weights_from(ref)
    for L0, La, Lb in zip(ref.layers, a.layers, b.layers):
        for key in ("wqkv", "wo", "w13", "w2"):
            assert torch.equal(a.canonical(La, key), ref.canonical(L0, key))
            assert torch.equal(b.canonical(Lb, key), ref.canonical(L0, key))
        assert torch.equal(La["wo_d"], L0["wo_d"])  # a's decode copies were rebuilt from the new weights


@pytest.mark.parametrize("model", ["llama-tiny-d128", "mixtral-tiny-d128"])
def test_checkpoint_roundtrip_into_one_layout(monkeypatch, tmp_path, model):
    """A checkpoint saved from the row-major model loads into a ONE_LAYOUT model: the derived
    tensors are dropped before the new ones arrive, the weights are packed again, and the model
    computes what the source does."""
    from k8s_llm_monitor_amd.models.checkpoint import load_checkpoint, save_checkpoint

    ref, one = _pair(monkeypatch, model)
    cfg = get_config(model)
    monkeypatch.setattr(CausalLM, "ONE_LAYOUT", False)
    src = CausalLM(cfg, device="cpu", dtype=torch.float32, seed=77)
    save_checkpoint(src, tmp_path)
    monkeypatch.setattr(CausalLM, "ONE_LAYOUT", "force")
    load_checkpoint(one, tmp_path)
    assert one._packed and one.layers[0]["w13"].dim() == (5 if cfg.is_moe else 4) and one.lm_head is one.lm_head_d
    for L, L0 in zip(one.layers, src.layers):
        for key in ("wqkv", "wo", "w13", "w2"):
            assert torch.equal(one.canonical(L, key), src.canonical(L0, key))
    x = torch.randn(5, cfg.d_model)
    assert (one._logits(x) - src._logits(x)).abs().max().item() < 1e-4


def test_moe_grouped_gemm_packed_cpu_path():
    """ops.moe_grouped_gemm over fragment-packed expert weights (ONE_LAYOUT) equals the row-major
    form: plain, and SwiGLU over the per-16 gate / up pairing (swiglu=8) vs the per-128 one."""
    torch.manual_seed(3)
    E, F, d = 3, 128, 64
    x = torch.randn(20, d)
    w13 = torch.randn(E, 2 * F, d) * 0.1  # [gate; up] per expert
    off = torch.tensor([2, 9, 9, 20], dtype=torch.int32)  # rows 0-1 belong to another rank
    w_il = torch.stack([ops.interleave_gate_up(w) for w in w13])
    w_pk = torch.stack([ops.pack_skinny(ops.interleave_gate_up8(w)) for w in w13])
    a = ops.moe_grouped_gemm(x, w_il, off, swiglu=True)
    b = ops.moe_grouped_gemm(x, w_pk, off, swiglu=8)
    assert torch.equal(b[:2], torch.zeros(2, F))
    torch.testing.assert_close(a, b, atol=1e-5, rtol=1e-5)
    w2 = torch.randn(E, d, F) * 0.1
    h = torch.randn(20, F)
    torch.testing.assert_close(ops.moe_grouped_gemm(h, w2, off),
                               ops.moe_grouped_gemm(h, torch.stack([ops.pack_skinny(w) for w in w2]), off),
                               atol=1e-5, rtol=1e-5)
