"""The shared-A decode GEMM (gemm_decode.hip: packed weight streamed into registers, A staged in LDS
once per workgroup and shared by waves that split the columns) against an fp32 reference of the
same product, for every epilogue the decode path uses (split-K slabs, bf16 LM head, packed SwiGLU
over the [8 gate | 8 up] weight), with and without the deferred RMSNorm row scale, at Llama-3-8B
projection shapes and at every row count class (1 m-tile .. 4 m-tiles, ragged)."""
import pytest
import torch

from k8s_llm_monitor_amd import ops

pytestmark = pytest.mark.gpu
DEV = "cuda"
F_ = torch.nn.functional


@pytest.fixture(autouse=True, scope="module")
def _native_loaded():
    ops.native()
    torch.manual_seed(0)


def _check(y, ref, what, tol=2.5e-2):
    err = (y.float() - ref.float()).abs().max().item()
    scale = ref.float().abs().max().item()
    assert err <= tol * scale + 1e-3, f"{what}: max err {err:.4g} vs scale {scale:.4g}"


def _w(N, K, s=0.02):
    return (torch.randn(N, K, device=DEV, dtype=torch.bfloat16) * s).to(torch.bfloat16)


CASES = [  # (N, K, cfg)  - the engine's picks plus ragged / edge configurations
    (6144, 4096, (4, 1, 6, 8)),  # the engine's qkv pick: 6-wave workgroups
    (6144, 4096, (8, 1, 8, 8)),
    (4096, 4096, (8, 1, 8, 8)),
    (4096, 4096, (4, 1, 4, 16)),
    (4096, 14336, (8, 1, 8, 8)),
    (4096, 14336, (4, 1, 4, 16)),
    (1024, 512, (2, 1, 4, 8)),
    (320, 1024, (1, 1, 8, 8)),  # 20 n-tiles, 8 per workgroup: the third workgroup is ragged
    (1280, 8192, (16, 1, 4, 16)),  # Llama-3-70B qkv at TP=8
]


@pytest.mark.parametrize("M", [1, 17, 40, 64])
@pytest.mark.parametrize("N,K,cfg", CASES)
def test_dec_slabs_match_fp32(M, N, K, cfg):
    x = torch.randn(M, K, device=DEV, dtype=torch.bfloat16)
    w = _w(N, K)
    ws = torch.empty(cfg[0] * M * N, device=DEV, dtype=torch.float32)
    s = ops.dec_gemm(ops.pack_activation(x), ops.pack_skinny(w), 0, M, workspace=ws, cfg=cfg)
    assert s == cfg[0]
    y = ws[: s * M * N].view(s, M, N).sum(0)
    _check(y, x.float() @ w.float().t(), f"slabs M{M} N{N} K{K} cfg{cfg}")
    # every slab is the product over its own K slice
    kc = K // s
    last = x[:, (s - 1) * kc:].float() @ w[:, (s - 1) * kc:].float().t()
    _check(ws[(s - 1) * M * N: s * M * N].view(M, N), last, "last slab")


@pytest.mark.parametrize("M", [1, 33, 64])
def test_dec_rownorm_scale(M):
    """Deferred RMSNorm: A holds x * w; outputs scaled by 1/rms from add_norm_partial's sums."""
    N, K = 4096, 4096
    res = torch.randn(M, K, device=DEV, dtype=torch.bfloat16)
    nw = (torch.rand(K, device=DEV) + 0.5).to(torch.bfloat16)
    w = _w(N, K)
    xw, ss = ops.add_norm_partial(res.clone(), None, 0, nw)
    ws = torch.empty(8 * M * N, device=DEV, dtype=torch.float32)
    s = ops.dec_gemm(xw, ops.pack_skinny(w), 0, M, workspace=ws, rownorm=(ss, 1e-5), cfg=(8, 1, 8, 8))
    y = ws[: s * M * N].view(s, M, N).sum(0)
    xn = F_.rms_norm(res.float(), (K,), nw.float(), 1e-5)
    _check(y, xn @ w.float().t(), f"rownorm M{M}", tol=3e-2)


@pytest.mark.parametrize("M", [1, 20, 64])
@pytest.mark.parametrize("cfg", [(1, 1, 7, 16), (1, 1, 8, 16), (1, 1, 7, 8)])
def test_dec_swiglu8_feeds_down(M, cfg):
    K, F = 4096, 14336
    x = torch.randn(M, K, device=DEV, dtype=torch.bfloat16)
    wg, wu = _w(F, K), _w(F, K)
    act = ops.packed_empty(M, F, torch.bfloat16, DEV)
    ops.dec_gemm(ops.pack_activation(x), ops.pack_skinny(ops.interleave_gate_up8(torch.cat([wg, wu]))), 2, M,
                 out=act, cfg=cfg)
    g = (x.float() @ wg.float().t()).to(torch.bfloat16).float()
    u = (x.float() @ wu.float().t()).to(torch.bfloat16).float()
    _check(ops.unpack_skinny(act)[:M], F_.silu(g) * u, f"swiglu8 M{M} cfg{cfg}")


@pytest.mark.parametrize("M", [1, 64])
@pytest.mark.parametrize("cfg", [(1, 4, 8, 4), (1, 3, 8, 8), (1, 2, 8, 8)])
def test_dec_bf16_lm_head(M, cfg):
    """LM-head shape: N = 128256 does not divide the workgroup tile - the last workgroup is ragged."""
    N, K = 128256, 4096
    x = torch.randn(M, K, device=DEV, dtype=torch.bfloat16)
    w = _w(N, K)
    y = torch.full((M, N), float("nan"), device=DEV, dtype=torch.bfloat16)
    ops.dec_gemm(ops.pack_activation(x), ops.pack_skinny(w), 1, M, out=y, cfg=cfg)
    ref = x.float() @ w.float().t()
    _check(y, ref, f"lm_head M{M} cfg{cfg}")
    assert not torch.isnan(y).any(), "every column written (the ragged last workgroup included)"


@pytest.mark.parametrize("M", [1, 64])
@pytest.mark.parametrize("N", [32000, 16032])
def test_dec_bf16_head_one_tile_per_wave(M, N):
    """Mixtral's head (32000 rows) and a TP=8 vocab shard on the 8-wave one-tile config (1, 1, 8, 8)."""
    K = 4096
    x = torch.randn(M, K, device=DEV, dtype=torch.bfloat16)
    w = _w(N, K)
    y = torch.full((M, N), float("nan"), device=DEV, dtype=torch.bfloat16)
    ops.dec_gemm(ops.pack_activation(x), ops.pack_skinny(w), 1, M, out=y, cfg=(1, 1, 8, 8))
    _check(y, x.float() @ w.float().t(), f"head N{N} M{M}")
    assert not torch.isnan(y).any()


@pytest.mark.parametrize("M", [1, 23, 64])
@pytest.mark.parametrize("E,F,d", [(2, 14336, 4096), (4, 1024, 512)])
def test_dec_grouped_experts_match_fp32(M, E, F, d):
    """The MoE decode MLP on the grouped shared-A GEMM (grid.z = expert):
    gate_up + SwiGLU of every expert over the shared rows, then the experts' down projections into
    slabs scaled by the routing weights - their sum is the expert combine.  Against fp32."""
    x = torch.randn(M, d, device=DEV, dtype=torch.bfloat16)
    w13 = [torch.cat([_w(F, d), _w(F, d)]) for _ in range(E)]  # [gate; up] per expert
    w2 = [_w(d, F) for _ in range(E)]
    wg = torch.stack([ops.pack_skinny(ops.interleave_gate_up8(w)) for w in w13])
    wd = torch.stack([ops.pack_skinny(w) for w in w2])
    rw = torch.rand(M, E, device=DEV)
    rw[rw < 0.5] = 0.0  # rows that skipped an expert
    act = torch.empty((E, -(-M // 16), 2 * F // 64, 64, 8), device=DEV, dtype=torch.bfloat16)
    ops.dec_gemm_grouped(ops.pack_activation(x), wg, 2, M, out=act)
    ws = torch.full((E * M * d,), float("nan"), device=DEV, dtype=torch.float32)
    ns = ops.dec_gemm_grouped(act, wd, 0, M, workspace=ws, row_w=rw)
    assert ns == E
    y = ws[: ns * M * d].view(ns, M, d).sum(0)
    ref = torch.zeros(M, d, device=DEV)
    for e in range(E):
        g = (x.float() @ w13[e][:F].float().t()).to(torch.bfloat16).float()
        u = (x.float() @ w13[e][F:].float().t()).to(torch.bfloat16).float()
        h = (F_.silu(g) * u).to(torch.bfloat16).float()
        _check(ops.unpack_skinny(act[e])[:M], h, f"grouped swiglu e{e} M{M}")
        ref += (h @ w2[e].float().t()) * rw[:, e:e + 1]
    _check(y, ref, f"grouped down + combine M{M} E{E}")


@pytest.mark.parametrize("M", [1, 37, 64])
def test_embed_norm_partial_matches_resolve_embed_norm(M):
    """The decode front end in one launch (embed_norm_partial) equals resolve_ids -> embedding ->
    add_norm_partial(nslabs=0): residual rows, packed residual * w, per-512-column sums of squares."""
    V, d = 1000, 4096
    emb = torch.randn(V, d, device=DEV, dtype=torch.bfloat16)
    nw = (torch.rand(d, device=DEV) + 0.5).to(torch.bfloat16)
    ids = torch.randint(0, V, (M,), device=DEV, dtype=torch.int32)
    prev = torch.randint(0, V, (64,), device=DEV, dtype=torch.int32)
    src = torch.where(torch.rand(M, device=DEV) < 0.5, torch.randint(0, 64, (M,), device=DEV),
                      torch.full((M,), -1, device=DEV)).to(torch.int32)
    res, xw, ss = ops.embed_norm_partial(ids, emb, nw, src, prev)
    rid = ops.resolve_ids(ids, src, prev)
    r0 = ops.embedding(rid, emb)
    xw0, ss0 = ops.add_norm_partial(r0.clone(), None, 0, nw)
    assert torch.equal(res, r0)
    assert torch.equal(ops.unpack_skinny(xw)[:M], ops.unpack_skinny(xw0)[:M])
    torch.testing.assert_close(ss, ss0, rtol=1e-5, atol=1e-4)


@pytest.mark.parametrize("M", [1, 17, 40, 64])
def test_dec_rc_matches_slabs_and_norm(M):
    """ops.dec_gemm_rc (row-complete o projection: residual add + deferred-norm operands in its
    epilogue) against the slab path (gemm_dec 8 split-K slabs + add_norm_partial): the residual and
    the normed A operand BIT-identical (same K slices summed in the same order), the per-16-column
    sums of squares equal to the per-512-column ones summed, and the gate_up GEMM that consumes
    them (wide 256-partial row scale) within rounding of the narrow form and of fp32."""
    d, F, eps = 4096, 14336, 1e-5
    g = torch.Generator(device=DEV).manual_seed(M)
    x = torch.randn(M, d, device=DEV, generator=g).to(torch.bfloat16)
    w = (torch.randn(d, d, device=DEV, generator=g) * 0.02).to(torch.bfloat16)
    wp = ops.pack_skinny(w)
    resid0 = torch.randn(M, d, device=DEV, generator=g).to(torch.bfloat16)
    nw = (1 + 0.1 * torch.randn(d, device=DEV, generator=g)).to(torch.bfloat16)
    xp = ops.pack_activation(x)
    for _ in range(3):  # repeated launches on the same buffers
        r_rc = resid0.clone()
        xw_rc, (ss_rc, _) = ops.dec_gemm_rc(xp, wp, M, r_rc, nw, eps)
        ws = torch.empty(8 * M * d, device=DEV)
        ns = ops.dec_gemm(xp, wp, 0, M, workspace=ws, cfg=(8, 1, 8, 8))
        r_sl = resid0.clone()
        xw_sl, ss_sl = ops.add_norm_partial(r_sl, ws, ns, nw)
        torch.cuda.synchronize()
        assert torch.equal(r_rc, r_sl)
        assert torch.equal(ops.unpack_skinny(xw_rc)[:M], ops.unpack_skinny(xw_sl)[:M])
        torch.testing.assert_close(ss_rc.view(M, 8, 32).sum(-1), ss_sl, rtol=1e-4, atol=1e-3)
    # consumer: gate_up + SwiGLU with the wide row scale
    w13 = (torch.randn(2 * F, d, device=DEV, generator=g) * 0.02).to(torch.bfloat16)
    w13p = ops.pack_skinny(ops.interleave_gate_up8(w13))
    a_rc = ops.packed_empty(M, F, torch.bfloat16, DEV)
    a_sl = ops.packed_empty(M, F, torch.bfloat16, DEV)
    ops.dec_gemm(xw_rc, w13p, 2, M, out=a_rc, rownorm=(ss_rc, eps))
    ops.dec_gemm(xw_sl, w13p, 2, M, out=a_sl, rownorm=(ss_sl, eps))
    _check(ops.unpack_skinny(a_rc)[:M], ops.unpack_skinny(a_sl)[:M].float(), f"rc vs slab gate_up M{M}", tol=1e-2)
    h = r_rc.float()
    xn = h * torch.rsqrt((h * h).mean(-1, keepdim=True) + eps) * nw.float()
    gu = xn @ w13.float().t()
    ref = F_.silu(gu[:, :F].to(torch.bfloat16).float()) * gu[:, F:].to(torch.bfloat16).float()
    _check(ops.unpack_skinny(a_rc)[:M], ref, f"rc gate_up vs fp32 M{M}")


