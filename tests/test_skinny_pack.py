"""Host-side layout helpers of the decode skinny GEMM (the GPU numerics are in test_ops_gpu.py)."""
import pytest
import torch

from k8s_llm_monitor_amd import ops


def test_pack_roundtrip_and_fragment_order():
    N, K = 48, 96
    w = torch.arange(N * K, dtype=torch.float32).reshape(N, K)
    wp = ops.pack_skinny(w)
    assert wp.shape == (N // 16, K // 32, 64, 8)
    assert torch.equal(ops.unpack_skinny(wp), w)
    # block (j, s), lane l = 16 q + r holds W[16 j + r, 32 s + 8 q : +8]
    j, s, q, r = 2, 1, 3, 5
    assert torch.equal(wp[j, s, 16 * q + r], w[16 * j + r, 32 * s + 8 * q: 32 * s + 8 * q + 8])


def test_interleave_gate_up():
    F, K = 128, 32
    g = torch.full((F, K), 1.0)
    u = torch.full((F, K), 2.0)
    g[:, 0] = torch.arange(F)
    u[:, 0] = torch.arange(F)
    w = ops.interleave_gate_up(torch.cat([g, u]))
    # tile t (128 rows) = gate rows 64t..64t+63 then up rows 64t..64t+63
    assert torch.equal(w[:64, 1], torch.ones(64)) and torch.equal(w[64:128, 1], torch.full((64,), 2.0))
    assert torch.equal(w[128:192, 0], torch.arange(64, 128, dtype=torch.float32))


def test_deinterleave_and_interleaved_silu_mul():
    """The single resident w13 is gate/up-interleaved: de-interleaving restores [gate; up], and
    silu_mul over the interleaved GEMM output equals silu_mul over the canonical one."""
    F, K = 192, 16
    w = torch.randn(2 * F, K)
    wi = ops.interleave_gate_up(w)
    assert torch.equal(ops.deinterleave_gate_up(wi), w)
    x = torch.randn(5, K)
    y_can = ops.silu_mul(x @ w.t())
    y_il = ops.silu_mul(x @ wi.t(), interleaved=True)
    assert torch.allclose(y_can, y_il, atol=1e-6)


def test_model_single_weight_copy_cpu():
    """Row-major layout: the decode-path weight views ARE the prefill tensors (no second copy)."""
    from k8s_llm_monitor_amd.models.config import get_config
    from k8s_llm_monitor_amd.models.llama import CausalLM

    m = CausalLM(get_config("llama-tiny"), device="cpu", dtype=torch.float32, seed=1)
    if m.skinny_layout != "rowmajor":
        pytest.skip("tiny config not eligible for the row-major skinny path")
    L = m.layers[0]
    assert L["wqkv_p"] is L["wqkv"] and L["wo_p"] is L["wo"] and L["w13_p"] is L["w13"] and L["w2_p"] is L["w2"]


def test_skinny_splits_bounds(monkeypatch):
    monkeypatch.setattr(ops, "SKINNY_SPLITS_FORCE", 0)
    assert ops.skinny_splits(4096, 4096) == 4
    assert ops.skinny_splits(4096, 14336) == 4
    assert ops.skinny_splits(6144, 4096) == 3
    assert ops.skinny_splits(64, 256) == 1
    monkeypatch.setattr(ops, "SKINNY_SPLITS_FORCE", 3)
    assert ops.skinny_splits(4096, 4096) == 3


def test_skinny_auto_splits_whole_rounds(monkeypatch):
    """Automatic split-K (mirror of the HIP launcher): power of two, grid <= one workgroup per CU,
    slices >= 512 deep and a multiple of the 4 waves' 256-deep round."""
    assert ops.skinny_auto_splits(64, 6144, 4096) == 2   # Llama-3-8B qkv: 96 tiles x 2
    assert ops.skinny_auto_splits(64, 4096, 4096) == 4   # o
    assert ops.skinny_auto_splits(64, 4096, 14336) == 4  # down
    assert ops.skinny_auto_splits(64, 1280, 8192) == 8   # Llama-3-70B qkv at TP=8
    assert ops.skinny_auto_splits(64, 256, 128) == 1     # tiny model: no split
    for N, K in ((6144, 4096), (4096, 14336), (1280, 8192), (28672, 4096)):
        s = ops.skinny_auto_splits(64, N, K)
        assert s == 1 or ((N // 64) * s <= 256 and K % (s * 256) == 0)


@pytest.mark.parametrize("model", ["llama-tiny-d128", "mixtral-tiny-d128"])
def test_decode_skinny_path_matches_generic_cpu(monkeypatch, model):
    """The decode control flow over packed weights (split-K slabs reduced in rope / the norm tail;
    SwiGLU epilogue) equals the generic path, on the CPU forms of the ops (fp32)."""
    from k8s_llm_monitor_amd.models import AttnMeta, CausalLM, get_config

    monkeypatch.setattr(ops, "SKINNY_SPLITS_FORCE", 3)  # force real split-K slicing on tiny shapes
    cfg = get_config(model)
    m = CausalLM(cfg, device="cpu", dtype=torch.float32, seed=3)
    assert m._skinny_ws is not None and m._split_d == 3
    monkeypatch.setattr(ops, "SKINNY_SPLITS_FORCE", 0)
    m0 = CausalLM(cfg, device="cpu", dtype=torch.float32, seed=3)
    assert m0._split_d == 0  # automatic split-K per call
    B, bs, nb = 3, 16, 8
    g = torch.Generator().manual_seed(0)
    kv = [(torch.randn(nb, m.hkv, m.D // 8, bs, 8, generator=g), torch.randn(nb, m.hkv, m.D, bs, generator=g))
          for _ in m.layers]
    lens = torch.tensor([3, 17, 9], dtype=torch.int32)
    meta = AttnMeta(is_prefill=False, positions=lens - 1, slot_mapping=torch.full((B,), -1, dtype=torch.int32),
                    block_tables=torch.arange(B * 2, dtype=torch.int32).view(B, 2) % nb, seq_lens=lens)
    ids = torch.tensor([5, 77, 300], dtype=torch.int32)
    a = m.forward(ids, meta, kv)
    monkeypatch.setattr(CausalLM, "SKINNY_DECODE", False)
    b = m.forward(ids, meta, kv)
    assert (a - b).abs().max().item() < 1e-4


def test_moe_grouped_gemm_cpu_path():
    """CPU form of the grouped expert GEMM: per-expert row blocks from the offsets, SwiGLU over the
    interleaved w13, rows outside the offset range untouched (zero)."""
    counts = [3, 0, 5]
    x = torch.randn(sum(counts) + 2, 64)
    w = torch.randn(3, 128, 64)
    off = torch.tensor([2, 5, 5, 10], dtype=torch.int32)  # rows 0-1 belong to another rank
    y = ops.moe_grouped_gemm(x, w, off)
    assert torch.equal(y[:2], torch.zeros(2, 128))
    assert torch.allclose(y[2:5], x[2:5] @ w[0].t(), atol=1e-5)
    assert torch.allclose(y[5:10], x[5:10] @ w[2].t(), atol=1e-5)
    wi = torch.stack([ops.interleave_gate_up(e) for e in w])
    ys = ops.moe_grouped_gemm(x, wi, off, swiglu=True)
    g, u = (x[5:10] @ w[2].t()).chunk(2, dim=1)
    assert torch.allclose(ys[5:10], torch.nn.functional.silu(g) * u, atol=1e-4)


def test_gemm_tile_cpu_path():
    """ops.gemm_tile off the GPU: dense, grouped (rows outside the offsets stay zero) and SwiGLU
    against plain fp32 references (the HIP numerics are in test_gemm_tile_gpu.py)."""
    F_ = torch.nn.functional
    torch.manual_seed(0)
    x = torch.randn(37, 64)
    w = torch.randn(256, 64) * 0.1
    torch.testing.assert_close(ops.gemm_tile(x, w), F_.linear(x, w))
    we = torch.randn(3, 256, 64) * 0.1
    off = torch.tensor([5, 10, 10, 30], dtype=torch.int32)  # experts 0..2 own rows 5..29
    y = ops.gemm_tile(x, we, off)
    assert torch.all(y[:5] == 0) and torch.all(y[30:] == 0)
    torch.testing.assert_close(y[5:10], F_.linear(x[5:10], we[0]))
    torch.testing.assert_close(y[10:30], F_.linear(x[10:30], we[2]))
    wi = ops.interleave_gate_up(we[1])
    torch.testing.assert_close(ops.gemm_tile(x, wi, swiglu=True),
                               ops.silu_mul(F_.linear(x, we[1]), interleaved=False))


def test_gemm_tile_rope_cpu_path():
    """ops.gemm_tile(rope=...) off the GPU rotates heads 0 .. heads - 1 of the bf16 product exactly as
    ops.reference.apply_rope and leaves the rest; rejected with grouped / SwiGLU weights."""
    from k8s_llm_monitor_amd.ops import reference as ref

    torch.manual_seed(3)
    M, K, H, Hr = 40, 256, 6, 4
    x = torch.randn(M, K, dtype=torch.bfloat16)
    w = (torch.randn(H * 128, K) * 0.05).to(torch.bfloat16)
    cs = ref.rope_cos_sin(512, 128, 10000.0)
    pos = torch.randint(0, 512, (M,), dtype=torch.int32)
    y = ops.gemm_tile(x, w, rope=(pos, cs, Hr))
    plain = torch.nn.functional.linear(x.float(), w.float()).to(torch.bfloat16)
    want = ref.apply_rope(plain[:, : Hr * 128].view(M, Hr, 128), pos, cs).reshape(M, -1)
    torch.testing.assert_close(y[:, : Hr * 128].float(), want, atol=2e-2, rtol=1e-2)
    assert torch.equal(y[:, Hr * 128:], plain[:, Hr * 128:])
    # the routing entry point reports that the library took it (RoPE left to rope_and_cache)
    y2, rotated = ops.prefill_linear(x, w, rope=(pos, cs, Hr))
    assert not rotated
    torch.testing.assert_close(y2.float(), plain.float(), atol=2e-2, rtol=1e-2)
    import pytest
    with pytest.raises(ValueError):
        ops.gemm_tile(x, w, swiglu=True, rope=(pos, cs, Hr))


def test_fused_norm_epilogues_cpu_path():
    """gemm_tile_resid (residual add + next RMSNorm's weighted input + per-128-column sums of
    squares) followed by gemm_tile(rowscale=...) equals rms_norm(resid + x W^T) * w projected -
    the CPU reference of the fused prefill norm (HIP numerics: test_tile_real_shapes_gpu.py)."""
    from k8s_llm_monitor_amd.ops import reference as ref

    torch.manual_seed(5)
    M, d, F = 64, 256, 512
    x = torch.randn(M, d, dtype=torch.bfloat16)
    wo = (torch.randn(d, d) * 0.05).to(torch.bfloat16)
    res = torch.randn(M, d, dtype=torch.bfloat16)
    nw = (torch.rand(d) + 0.5).to(torch.bfloat16)
    w13 = (torch.randn(2 * F, d) * 0.05).to(torch.bfloat16)
    r0 = res.clone()
    hw, ss = ops.gemm_tile_resid(x, wo, res, nw)
    h = (torch.nn.functional.linear(x.float(), wo.float()).to(torch.bfloat16).float() + r0.float()).to(torch.bfloat16)
    assert torch.equal(res, h)
    torch.testing.assert_close(ss.sum(1), (h.float() ** 2).sum(1), rtol=1e-5, atol=1e-3)
    y = ops.gemm_tile(hw, ops.interleave_gate_up(w13), swiglu=True, rowscale=(ss, 1e-5))
    xn = ref.rms_norm(h, nw, 1e-5)
    want = ops.silu_mul(torch.nn.functional.linear(xn.float(), w13.float()).to(torch.bfloat16))
    torch.testing.assert_close(y.float(), want.float(), atol=3e-2, rtol=3e-2)
    import pytest
    with pytest.raises(ValueError):
        ops.gemm_tile(hw, wo, rowscale=(ss, 1e-5))  # only the fused consumers take a row scale


def test_embed_norm_partial_cpu_path():
    """ops.embed_norm_partial off the GPU = resolve_ids -> embedding -> add_norm_partial(nslabs=0)."""
    torch.manual_seed(7)
    V, d, M = 50, 512, 5
    emb = torch.randn(V, d, dtype=torch.bfloat16)
    nw = (torch.rand(d) + 0.5).to(torch.bfloat16)
    ids = torch.tensor([3, 7, 11, 13, 17], dtype=torch.int32)
    prev = torch.tensor([40, 41, 42], dtype=torch.int32)
    src = torch.tensor([-1, 2, -1, 0, -1], dtype=torch.int32)
    res, xw, ss = ops.embed_norm_partial(ids, emb, nw, src, prev)
    want_ids = torch.tensor([3, 42, 11, 40, 17])
    assert torch.equal(res, emb[want_ids])
    xw0, ss0 = ops.add_norm_partial(emb[want_ids].clone(), None, 0, nw)
    assert torch.equal(xw, xw0) and torch.allclose(ss, ss0)
