"""Numerics of every gfx950 HIP kernel against the plain-PyTorch fp32 reference of the same op."""
import math

import pytest
import torch

from k8s_llm_monitor_amd import ops
from k8s_llm_monitor_amd.ops import reference as ref

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.fixture(autouse=True, scope="module")
def _native_loaded():
    ops.native()  # fail loudly when the extension is missing on a GPU box
    torch.manual_seed(0)


def _close(a, b, atol, rtol=0.0, what=""):
    err = (a.float() - b.float()).abs()
    tol = atol + rtol * b.float().abs()
    bad = (err > tol).sum().item()
    assert bad == 0, f"{what}: {bad} elements out of tolerance, max err {err.max().item():.4g}"


@pytest.mark.parametrize("rows,d", [(1, 4096), (64, 4096), (333, 8192), (7, 768), (5, 1024)])
def test_rms_norm(rows, d):
    x = torch.randn(rows, d, device=DEV, dtype=torch.bfloat16)
    w = torch.randn(d, device=DEV, dtype=torch.bfloat16)
    y = ops.rms_norm(x, w, 1e-5)
    _close(y, ref.rms_norm(x.cpu(), w.cpu(), 1e-5).to(DEV), atol=2e-2, rtol=1e-2, what="rms_norm")


@pytest.mark.parametrize("rows,d", [(64, 4096), (129, 8192)])
def test_fused_add_rms_norm(rows, d):
    x = torch.randn(rows, d, device=DEV, dtype=torch.bfloat16)
    r = torch.randn(rows, d, device=DEV, dtype=torch.bfloat16)
    w = torch.randn(d, device=DEV, dtype=torch.bfloat16)
    y_ref, s_ref = ref.fused_add_rms_norm(x.cpu(), r.cpu(), w.cpu(), 1e-5)
    y = ops.fused_add_rms_norm(x, r, w, 1e-5)
    _close(r, s_ref.to(DEV), atol=1e-2, rtol=1e-2, what="residual")
    _close(y, y_ref.to(DEV), atol=3e-2, rtol=1e-2, what="norm")


def test_layer_norm():
    x = torch.randn(37, 768, device=DEV, dtype=torch.bfloat16)
    w = torch.randn(768, device=DEV, dtype=torch.bfloat16)
    b = torch.randn(768, device=DEV, dtype=torch.bfloat16)
    _close(ops.layer_norm(x, w, b, 1e-5), ref.layer_norm(x.cpu(), w.cpu(), b.cpu(), 1e-5).to(DEV),
           atol=3e-2, rtol=1e-2, what="layer_norm")


@pytest.mark.parametrize("rows,F", [(1, 14336), (64, 14336), (300, 3584)])
def test_silu_mul(rows, F):
    x = torch.randn(rows, 2 * F, device=DEV, dtype=torch.bfloat16)
    _close(ops.silu_mul(x), ref.silu_mul(x.cpu()).to(DEV), atol=2e-2, rtol=1e-2, what="silu_mul")


def test_gelu():
    x = torch.randn(100, 3072, device=DEV, dtype=torch.bfloat16)
    _close(ops.gelu_tanh(x), ref.gelu_tanh(x.cpu()).to(DEV), atol=2e-2, rtol=1e-2, what="gelu")


def test_embedding_vocab_parallel():
    w = torch.randn(1000, 512, device=DEV, dtype=torch.bfloat16)
    ids = torch.randint(0, 2000, (77,), device=DEV, dtype=torch.int32)
    y = ops.embedding(ids, w, vocab_start=500)
    assert torch.equal(y.cpu(), ref.embedding(ids.cpu(), w.cpu(), 500))


def _make_cache(nb, hkv, d, bs=16):
    k = torch.randn(nb, hkv, d // 8, bs, 8, device=DEV, dtype=torch.bfloat16)
    v = torch.randn(nb, hkv, d, bs, device=DEV, dtype=torch.bfloat16)
    return k, v


@pytest.mark.parametrize("hq,hkv,d", [(32, 8, 128), (8, 8, 128), (64, 8, 128), (16, 4, 64)])
def test_rope_and_cache(hq, hkv, d):
    T, nb = 50, 16
    qkv = torch.randn(T, (hq + 2 * hkv) * d, device=DEV, dtype=torch.bfloat16)
    pos = torch.randint(0, 4000, (T,), device=DEV, dtype=torch.int32)
    cs = ref.rope_cos_sin(8192, d, 500000.0, device=DEV)
    slots = torch.randperm(nb * 16, device=DEV)[:T].to(torch.int32)
    slots[3] = -1  # padding token: no cache write
    kc, vc = _make_cache(nb, hkv, d)
    kc0, vc0 = kc.clone().cpu(), vc.clone().cpu()
    q2 = qkv.clone().cpu()
    ops.rope_and_cache(qkv, pos, cs, kc, vc, slots, hq, hkv, d)
    ref.rope_and_cache(q2, pos.cpu(), cs.cpu(), kc0, vc0, slots.cpu(), hq, hkv, d)
    _close(qkv, q2.to(DEV), atol=2e-2, rtol=1e-2, what="rope qkv")
    _close(kc, kc0.to(DEV), atol=2e-2, rtol=1e-2, what="k_cache")
    assert torch.equal(vc.cpu(), vc0), "v_cache"


@pytest.mark.parametrize("splits", [None, 1, 3, 16])
@pytest.mark.parametrize("B,hq,hkv,d,maxlen", [(1, 32, 8, 128, 33), (8, 32, 8, 128, 1100), (64, 32, 8, 128, 700),
                                                (3, 64, 8, 128, 2000), (5, 8, 8, 128, 300), (4, 16, 4, 64, 513),
                                                (2, 64, 8, 128, 5000)])
def test_paged_decode(B, hq, hkv, d, maxlen, splits):
    bs = 16
    max_blocks = (maxlen + bs - 1) // bs + 1
    nb = B * max_blocks + 4
    kc, vc = _make_cache(nb, hkv, d, bs)
    lens = torch.randint(1, maxlen + 1, (B,), dtype=torch.int32)
    lens[0] = maxlen
    perm = torch.randperm(nb)[: B * max_blocks].view(B, max_blocks).to(torch.int32)
    bt = perm.to(DEV)
    q = torch.randn(B, (hq + 2 * hkv) * d, device=DEV, dtype=torch.bfloat16)  # q inside fused rows
    scale = 1.0 / math.sqrt(d)
    y = ops.paged_decode(q, kc, vc, bt, lens.to(DEV), hq, hkv, d, scale, splits=splits)
    r = ref.paged_decode(q.cpu(), kc.cpu(), vc.cpu(), perm, lens, hq, hkv, d, scale)
    _close(y, r.to(DEV), atol=2e-2, rtol=2e-2, what="paged_decode")


def test_paged_decode_zero_len_rows():
    hq, hkv, d = 32, 8, 128
    kc, vc = _make_cache(64, hkv, d)
    bt = torch.arange(64, device=DEV, dtype=torch.int32).view(4, 16)
    lens = torch.tensor([0, 17, 0, 256], device=DEV, dtype=torch.int32)
    q = torch.randn(4, hq * d, device=DEV, dtype=torch.bfloat16)
    y = ops.paged_decode(q, kc, vc, bt, lens, hq, hkv, d, 0.088)
    assert torch.all(y[0] == 0) and torch.all(y[2] == 0)
    r = ref.paged_decode(q.cpu(), kc.cpu(), vc.cpu(), bt.cpu(), lens.cpu(), hq, hkv, d, 0.088)
    _close(y, r.to(DEV), atol=2e-2, rtol=2e-2, what="paged_decode pad rows")


@pytest.mark.parametrize("lens,hq,hkv,splits,nslabs", [([1, 2, 17, 256, 257, 1800], 32, 8, None, 2),
                                                        ([300, 77, 1024, 513], 32, 8, 4, 3),
                                                        ([40, 600], 64, 8, 2, 1), ([129, 64], 8, 8, None, 2)])
def test_paged_decode_fused_matches_rope_then_decode(lens, hq, hkv, splits, nslabs):
    """paged_decode_fused (slab reduce + RoPE + KV write + attention over cache + new token in
    one kernel) == rope_and_cache from the slabs, then paged_decode - outputs and cache contents."""
    d, bs = 128, 16
    B = len(lens)
    max_blocks = (max(lens) + bs - 1) // bs + 1
    nb = B * max_blocks + 4
    kc, vc = _make_cache(nb, hkv, d, bs)
    lens_t = torch.tensor(lens, dtype=torch.int32, device=DEV)
    bt = torch.randperm(nb, device=DEV)[: B * max_blocks].view(B, max_blocks).to(torch.int32)
    pos = lens_t - 1
    slots = torch.stack([bt[b, (lens[b] - 1) // bs] * bs + (lens[b] - 1) % bs for b in range(B)]).to(torch.int32)
    n = (hq + 2 * hkv) * d
    slabs = torch.randn(nslabs, B, n, device=DEV, dtype=torch.float32) * 0.5
    cs = ref.rope_cos_sin(4096, d, 500000.0, None, device=DEV)
    scale = 1.0 / math.sqrt(d)
    kc2, vc2 = kc.clone(), vc.clone()
    y = ops.paged_decode_fused(slabs.reshape(-1), nslabs, pos, cs, slots, kc, vc, bt, lens_t, hq, hkv, d, scale,
                               splits=splits)
    qkv = torch.empty(B, n, device=DEV, dtype=torch.bfloat16)
    ops.rope_and_cache(qkv, pos, cs, kc2, vc2, slots, hq, hkv, d, partial=slabs.reshape(-1), nslabs=nslabs)
    r = ops.paged_decode(qkv, kc2, vc2, bt, lens_t, hq, hkv, d, scale, splits=splits)
    _close(kc, kc2, atol=1e-2, rtol=1e-2, what="k cache")
    _close(vc, vc2, atol=1e-2, rtol=1e-2, what="v cache")
    _close(y, r, atol=2e-2, rtol=2e-2, what="fused decode vs rope + decode")
    rr = ref.paged_decode(qkv.cpu(), kc2.cpu(), vc2.cpu(), bt.cpu(), lens_t.cpu(), hq, hkv, d, scale)
    _close(y.cpu(), rr, atol=2e-2, rtol=2e-2, what="fused decode vs fp32 reference")


def test_paged_decode_fused_in_launch_merge_bit_identical():
    """The split partials merged by the last-arriving split inside the attention launch (write-
    through partials, one agent-scope counter per (sequence, kv head)) == the separate
    paged_decode_reduce launch, bit for bit - over back-to-back launches whose lengths change the
    number of valid splits each time, leaving every counter at zero."""
    d, bs, hq, hkv = 128, 16, 32, 8
    B, nslabs = 4, 2
    max_blocks = 2304 // bs + 1
    nb = B * max_blocks + 4
    kc, vc = _make_cache(nb, hkv, d, bs)
    bt = torch.randperm(nb, device=DEV)[: B * max_blocks].view(B, max_blocks).to(torch.int32)
    n = (hq + 2 * hkv) * d
    cs = ref.rope_cos_sin(4096, d, 500000.0, None, device=DEV)
    scale = 1.0 / math.sqrt(d)
    ws = ops.decode_workspace(B, hq, d, device=DEV, Hkv=hkv)
    ws_sep = (torch.empty_like(ws[0]), torch.empty_like(ws[1]))  # no counters: the two-launch path
    g = torch.Generator(device="cpu").manual_seed(7)
    for it, lens in enumerate([[1800, 5, 300, 2300], [40, 1999, 1, 257], [2300, 2300, 2300, 2300], [0, 700, 64, 1100],
                               [1800, 5, 300, 2300], [3, 4, 5, 6]]):
        for splits in (None, 16, 64):
            lens_t = torch.tensor(lens, dtype=torch.int32, device=DEV)
            pos = (lens_t - 1).clamp(min=0)
            slots = torch.stack([bt[b, max(lens[b] - 1, 0) // bs] * bs + max(lens[b] - 1, 0) % bs
                                 for b in range(B)]).to(torch.int32)
            slabs = (torch.randn(nslabs, B, n, generator=g) * 0.5).to(DEV)
            kc2, vc2 = kc.clone(), vc.clone()
            y = ops.paged_decode_fused(slabs.reshape(-1), nslabs, pos, cs, slots, kc, vc, bt, lens_t, hq, hkv, d,
                                       scale, workspace=ws, splits=splits)
            r = ops.paged_decode_fused(slabs.reshape(-1), nslabs, pos, cs, slots, kc2, vc2, bt, lens_t, hq, hkv, d,
                                       scale, workspace=ws_sep, splits=splits)
            torch.cuda.synchronize()
            live = [b for b in range(B) if lens[b] > 0]
            assert torch.equal(y[live], r[live]), f"launch {it} splits {splits}: merge != reduce launch"
            assert int(ws[2].abs().sum()) == 0, f"launch {it}: counters not reset"


@pytest.mark.parametrize("lens,hq,hkv", [([1], 32, 8), ([128], 32, 8), ([300, 77, 1024], 32, 8),
                                         ([513, 200], 64, 8), ([129, 64], 8, 8)])
def test_flash_prefill(lens, hq, hkv):
    d = 128
    T = sum(lens)
    qkv = torch.randn(T, (hq + 2 * hkv) * d, device=DEV, dtype=torch.bfloat16)
    cu = torch.tensor([0] + list(torch.tensor(lens).cumsum(0).tolist()), dtype=torch.int32, device=DEV)
    scale = 1.0 / math.sqrt(d)
    y = ops.flash_prefill(qkv, cu, hq, hkv, d, scale)
    r = ref.flash_prefill(qkv.cpu(), cu.cpu(), hq, hkv, d, scale)
    _close(y, r.to(DEV), atol=2e-2, rtol=2e-2, what="flash_prefill")


def test_flash_prefill_softmax_spike():
    """Force a large running-max jump mid-sequence (rescale branch) - rule 26."""
    hq, hkv, d, L = 8, 8, 128, 300
    qkv = torch.randn(L, (hq + 2 * hkv) * d, device=DEV, dtype=torch.bfloat16) * 0.1
    qkv[200, hq * d:(hq + hkv) * d] *= 400.0  # one key much larger than the rest
    cu = torch.tensor([0, L], dtype=torch.int32, device=DEV)
    y = ops.flash_prefill(qkv, cu, hq, hkv, d, 1 / math.sqrt(d))
    r = ref.flash_prefill(qkv.cpu(), cu.cpu(), hq, hkv, d, 1 / math.sqrt(d))
    _close(y, r.to(DEV), atol=3e-2, rtol=2e-2, what="flash_prefill spike")


@pytest.mark.parametrize("V", [128256, 32000, 50304])
def test_sample_greedy(V):
    logits = torch.randn(64, V, device=DEV, dtype=torch.bfloat16)
    logits[5, 1234] = 100.0
    tok = ops.sample(logits)
    assert torch.equal(tok.cpu(), ref.greedy(logits.cpu()))
    tok32 = ops.sample(logits.float())
    assert torch.equal(tok32.cpu(), ref.greedy(logits.cpu()))


def test_sample_topk_topp_temperature():
    B, V = 16, 32000
    logits = torch.randn(B, V, device=DEV, dtype=torch.float32) * 3
    temps = torch.full((B,), 0.7, device=DEV)
    topk = torch.full((B,), 5, device=DEV, dtype=torch.int32)
    topp = torch.ones(B, device=DEV)
    rng = torch.tensor([1234, 0], device=DEV, dtype=torch.int64)
    allowed = torch.topk(logits, 5, dim=-1).indices
    for i in range(20):
        rng[1] = i
        tok = ops.sample(logits, temps, topk, topp, rng).long()
        assert (allowed == tok[:, None]).any(-1).all(), "top-k violated"
    # top-p: with p small only the argmax survives
    topk.zero_()
    topp.fill_(1e-6)
    tok = ops.sample(logits, temps, topk, topp, rng)
    assert torch.equal(tok.cpu(), ref.greedy(logits.cpu()))


def test_sample_distribution():
    """Gumbel-max must sample softmax(logits/T): empirical frequencies over 4 tokens."""
    V = 4
    base = torch.tensor([0.0, 1.0, 2.0, 0.5])
    B = 4096
    logits = base.repeat(B, 1).to(DEV)
    temps = torch.full((B,), 1.0, device=DEV)
    rng = torch.tensor([7, 3], device=DEV, dtype=torch.int64)
    tok = ops.sample(logits, temps, None, None, rng).cpu()
    freq = torch.bincount(tok.long(), minlength=V).float() / B
    assert torch.allclose(freq, torch.softmax(base, 0), atol=0.03)


@pytest.mark.parametrize("T", [0.1, 0.7, 1.0, 3.0])
def test_sample_split_and_whole_row_paths_agree(T):
    """The split partial / final kernels and the whole-row (filtered) path draw the same Gumbel noise:
    with top_k = V - 1 (drops only the smallest logit) both must pick the same token (the noise is
    finite for every hash value, so no arbitrary element can win by an infinite draw)."""
    B, V = 64, 128256
    logits = (torch.randn(B, V, device=DEV) * 1.3).to(torch.bfloat16)
    temps = torch.full((B,), T, device=DEV)
    rng = torch.tensor([99, 7], device=DEV, dtype=torch.int64)
    fast = ops.sample(logits, temps, None, None, rng)
    full = ops.sample(logits, temps, torch.full((B,), V - 1, device=DEV, dtype=torch.int32), None, rng)
    assert torch.equal(fast, full)


def test_sample_advances_rng_in_kernel_and_graph():
    """advance=True bumps rng[1] inside the final sampling kernel: eager and hipGraph replays draw
    a fresh counter each time (the engine no longer launches a separate increment)."""
    B, V = 8, 32000
    logits = torch.randn(B, V, device=DEV)
    temps = torch.full((B,), 1.0, device=DEV)
    rng = torch.tensor([11, 5], device=DEV, dtype=torch.int64)
    a = ops.sample(logits, temps, None, None, rng, advance=True).clone()
    assert int(rng[1]) == 6 and int(rng[0]) == 11
    out = torch.empty(B, dtype=torch.int32, device=DEV)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        ops.sample(logits, temps, None, None, rng, out=out, advance=True)  # warm-up allocation
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        ops.sample(logits, temps, None, None, rng, out=out, advance=True)
    rng[1] = 5
    draws = []
    for _ in range(3):
        g.replay()
        draws.append(out.clone())
    torch.cuda.synchronize()
    assert int(rng[1]) == 8
    assert torch.equal(draws[0], a)  # replay 1 drew with counter 5, like the eager call
    assert not (torch.equal(draws[0], draws[1]) and torch.equal(draws[1], draws[2]))


def test_moe_route_align_combine():
    T, E, K, d = 300, 8, 2, 256
    logits = torch.randn(T, E, device=DEV)
    ids, w = ops.moe_route(logits, K, True)
    rids, rw = ref.moe_route(logits.cpu(), K, True)
    assert torch.equal(ids.cpu(), rids)
    assert torch.allclose(w.cpu(), rw, atol=1e-5)
    off, srt, inv = ops.moe_align(ids, E)
    roff, rsrt, rinv = ref.moe_align(ids.cpu(), E)
    assert torch.equal(off.cpu(), roff) and torch.equal(srt.cpu(), rsrt) and torch.equal(inv.cpu(), rinv)
    x = torch.randn(T, d, device=DEV, dtype=torch.bfloat16)
    xs = ops.gather_rows(x, srt, K)
    assert torch.equal(xs.cpu(), x.cpu()[srt.cpu().long() // K])
    y = ops.moe_combine(xs, inv, w, T)
    _close(y, ref.moe_combine(xs.cpu(), inv.cpu(), w.cpu(), T).to(DEV), atol=2e-2, rtol=1e-2, what="combine")


@pytest.mark.parametrize("splits", [1, 4, 7])
@pytest.mark.parametrize("M,N,K", [(1, 256, 512), (7, 4096, 4096), (16, 128, 1024), (33, 640, 14336),
                                   (64, 4096, 4096), (50, 6144, 4096)])
def test_gemm_skinny(M, N, K, splits):
    a = torch.randn(M, K, device=DEV, dtype=torch.bfloat16)
    w = (torch.randn(N, K, device=DEV, dtype=torch.bfloat16) * 0.05).to(torch.bfloat16)
    y = ops.gemm_skinny(a, w, splits=splits)
    y_ref = torch.nn.functional.linear(a.cpu().float(), w.cpu().float())
    _close(y.cpu(), y_ref, atol=3e-2, rtol=2e-2, what=f"gemm_skinny M{M} N{N} K{K} s{splits}")


@pytest.mark.parametrize("nt_tiles", [2, 4])
def test_gemm_skinny_nt_tiles(nt_tiles):
    a = torch.randn(24, 1024, device=DEV, dtype=torch.bfloat16)
    w = (torch.randn(96, 1024, device=DEV, dtype=torch.bfloat16) * 0.05).to(torch.bfloat16)
    if 96 % (16 * nt_tiles):
        pytest.skip("tile does not divide N")
    y = ops.skinny_linear(a, ops.pack_skinny(w), nt_tiles=nt_tiles)
    _close(y.cpu(), torch.nn.functional.linear(a.cpu().float(), w.cpu().float()), atol=3e-2, rtol=2e-2,
           what="nt_tiles")


@pytest.mark.parametrize("M", [1, 9, 64])
def test_skinny_swiglu(M):
    K, F = 1024, 448
    x = torch.randn(M, K, device=DEV, dtype=torch.bfloat16)
    w13 = (torch.randn(2 * F, K, device=DEV, dtype=torch.bfloat16) * 0.05).to(torch.bfloat16)
    act = ops.skinny_swiglu(x, ops.pack_skinny(ops.interleave_gate_up(w13)))
    gu = torch.nn.functional.linear(x.cpu().float(), w13.cpu().float()).to(torch.bfloat16)
    _close(act.cpu(), ref.silu_mul(gu), atol=3e-2, rtol=2e-2, what="swiglu")


@pytest.mark.parametrize("M", [1, 24, 64])
def test_proj_add_rms_norm(M):
    d, K = 4096, 1024
    a = torch.randn(M, K, device=DEV, dtype=torch.bfloat16)
    w = (torch.randn(d, K, device=DEV, dtype=torch.bfloat16) * 0.05).to(torch.bfloat16)
    r = torch.randn(M, d, device=DEV, dtype=torch.bfloat16)
    nw = torch.randn(d, device=DEV, dtype=torch.bfloat16)
    s_ref = (r.cpu().float() + torch.nn.functional.linear(a.cpu().float(), w.cpu().float())).to(torch.bfloat16)
    y_ref = ref.rms_norm(s_ref, nw.cpu(), 1e-5)
    y = ops.proj_add_rms_norm(a, ops.pack_skinny(w), r, nw, 1e-5, splits=4)
    _close(r.cpu(), s_ref, atol=3e-2, rtol=1e-2, what="residual")
    _close(y.cpu(), y_ref, atol=5e-2, rtol=2e-2, what="normed")


def test_rope_and_cache_from_slabs():
    """rope_and_cache reducing split-K qkv slabs == rope_and_cache on the summed bf16 qkv."""
    hq, hkv, D, T, S, bs = 32, 8, 128, 19, 5, 16
    ncol = (hq + 2 * hkv) * D
    part = torch.randn(S, T, ncol, device=DEV, dtype=torch.float32) * 0.3
    pos = torch.randint(0, 500, (T,), dtype=torch.int32, device=DEV)
    cs = ref.rope_cos_sin(2048, D, 500000.0, None, device=DEV)
    slots = torch.randperm(4 * bs, device=DEV)[:T].to(torch.int32)
    caches = [(torch.zeros(4, hkv, D // 8, bs, 8, device=DEV, dtype=torch.bfloat16),
               torch.zeros(4, hkv, D, bs, device=DEV, dtype=torch.bfloat16)) for _ in range(2)]
    qkv_a = torch.empty(T, ncol, device=DEV, dtype=torch.bfloat16)
    ops.rope_and_cache(qkv_a, pos, cs, caches[0][0], caches[0][1], slots, hq, hkv, D, partial=part.reshape(-1),
                       nslabs=S)
    qkv_b = part.sum(0).to(torch.bfloat16)
    ops.rope_and_cache(qkv_b, pos, cs, caches[1][0], caches[1][1], slots, hq, hkv, D)
    _close(qkv_a[:, : (hq + hkv) * D], qkv_b[:, : (hq + hkv) * D], atol=2e-2, rtol=1e-2, what="qk")
    _close(caches[0][0], caches[1][0], atol=2e-2, rtol=1e-2, what="k cache")
    _close(caches[0][1], caches[1][1], atol=2e-2, rtol=1e-2, what="v cache")


def test_llama_decode_skinny_matches_generic(monkeypatch):
    """The skinny decode tail (slab GEMMs + reduce kernels, deferred RMSNorm) and the hipBLASLt +
    fused_add_rms_norm path both match an fp32 CPU reference of the same decode step."""
    from k8s_llm_monitor_amd.models import AttnMeta, CausalLM, get_config

    cfg = get_config("llama-tiny-d128")
    m = CausalLM(cfg, device=DEV, seed=3)
    assert m._skinny_ws is not None
    B, bs = 5, 16
    nb = 2 * B  # no block shared between sequences (as the block manager guarantees for written blocks)
    kv = [(torch.randn(nb, m.hkv, m.D // 8, bs, 8, device=DEV, dtype=torch.bfloat16),
           torch.randn(nb, m.hkv, m.D, bs, device=DEV, dtype=torch.bfloat16)) for _ in m.layers]
    lens = torch.tensor([3, 17, 1, 30, 9], dtype=torch.int32, device=DEV)
    bt = torch.arange(B * 2, dtype=torch.int32, device=DEV).view(B, 2) % nb
    ids = torch.randint(0, cfg.vocab_size, (B,), dtype=torch.int32, device=DEV)
    # the new token's slot inside each sequence's last block (decode rows always write the cache;
    # the fused attention reads the new token from registers, the generic path from the cache)
    slots = torch.stack([bt[b, (int(lens[b]) - 1) // bs] * bs + (int(lens[b]) - 1) % bs for b in range(B)])
    meta = AttnMeta(is_prefill=False, positions=lens - 1, slot_mapping=slots.to(torch.int32),
                    block_tables=bt, seq_lens=lens,
                    decode_ws=ops.decode_workspace(B, m.hq, m.D, device=DEV, Hkv=m.hkv))
    kv0 = [(k.clone(), v.clone()) for k, v in kv]  # the caches before this step writes the new token
    a = m.forward(ids, meta, kv).float()
    monkeypatch.setattr(CausalLM, "SKINNY_DECODE", False)
    b = m.forward(ids, meta, kv).float()
    # fp32 CPU reference of the same decode step (same weights, the pre-step caches)
    rm = CausalLM(cfg, device="cpu", dtype=torch.float32, init="empty")
    rm.copy_weights_from(m)
    cpu = lambda t: t.cpu() if t is not None else None  # noqa: E731
    meta_c = AttnMeta(is_prefill=False, positions=cpu(meta.positions), slot_mapping=cpu(meta.slot_mapping),
                      block_tables=cpu(bt), seq_lens=cpu(lens))
    r = rm.forward(ids.cpu(), meta_c, [(k.float().cpu(), v.float().cpu()) for k, v in kv0]).float()
    scale = float(r.abs().max())
    for name, out in (("skinny", a), ("generic", b)):
        out = out.cpu()
        err = float((out - r).abs().max())
        assert err < 0.03 * scale, f"{name}: max-abs err {err:.4f} vs scale {scale:.3f}"
        # every row's argmax is the reference's or a provable near-tie (within 2x the bf16 error)
        got = r.gather(1, out.argmax(-1, keepdim=True)).squeeze(1)
        assert bool((r.max(-1).values - got <= 2 * err + 1e-6).all()), name


@pytest.mark.parametrize("M", [1, 17, 64])
def test_gemm_skinny_packed_activation(M):
    K, N = 1024, 256
    a = torch.randn(M, K, device=DEV, dtype=torch.bfloat16)
    w = (torch.randn(N, K, device=DEV, dtype=torch.bfloat16) * 0.05).to(torch.bfloat16)
    wp, ap = ops.pack_skinny(w), ops.pack_activation(a)
    y_ref = torch.nn.functional.linear(a.cpu().float(), w.cpu().float())
    _close(ops.skinny_linear(ap, wp, rows=M).cpu(), y_ref, atol=3e-2, rtol=2e-2, what="packed A, bf16 epi")
    ws = ops.skinny_workspace(M, N, 3, DEV)
    ns = ops.skinny_slabs(ap, wp, ws, 3, rows=M)
    _close(ops.reduce_slabs(ws, ns, M, N).cpu(), y_ref, atol=3e-2, rtol=2e-2, what="packed A, slabs")


@pytest.mark.parametrize("M", [3, 40])
def test_skinny_swiglu_packed_out_feeds_down(M):
    K, F, d = 512, 448, 256
    x = torch.randn(M, K, device=DEV, dtype=torch.bfloat16)
    w13 = (torch.randn(2 * F, K, device=DEV, dtype=torch.bfloat16) * 0.05).to(torch.bfloat16)
    w2 = (torch.randn(d, F, device=DEV, dtype=torch.bfloat16) * 0.05).to(torch.bfloat16)
    actp = ops.skinny_swiglu(ops.pack_activation(x), ops.pack_skinny(ops.interleave_gate_up(w13)), rows=M,
                             packed_out=True)
    gu = torch.nn.functional.linear(x.cpu().float(), w13.cpu().float()).to(torch.bfloat16)
    act_ref = ref.silu_mul(gu)
    _close(ops.unpack_skinny(actp)[:M].cpu(), act_ref, atol=3e-2, rtol=2e-2, what="packed act")
    y = ops.skinny_linear(actp, ops.pack_skinny(w2), rows=M)
    _close(y.cpu(), torch.nn.functional.linear(act_ref.float(), w2.cpu().float()), atol=5e-2, rtol=3e-2,
           what="down from packed act")


@pytest.mark.parametrize("M", [1, 21, 64])
def test_deferred_rmsnorm_chain(M):
    """add_norm_partial (residual += slabs; residual * w; partial sums of squares) followed by a
    skinny GEMM with rownorm == rms_norm(residual) @ W^T."""
    d, N, S = 4096, 512, 3
    r = torch.randn(M, d, device=DEV, dtype=torch.bfloat16)
    slabs = torch.randn(S, M, d, device=DEV, dtype=torch.float32) * 0.1
    nw = (torch.rand(d, device=DEV) + 0.5).to(torch.bfloat16)
    w = (torch.randn(N, d, device=DEV, dtype=torch.bfloat16) * 0.02).to(torch.bfloat16)
    r_ref = (r.cpu().float() + slabs.cpu().sum(0)).to(torch.bfloat16)
    x_ref = ref.rms_norm(r_ref, nw.cpu(), 1e-5)
    y_ref = torch.nn.functional.linear(x_ref.float(), w.cpu().float())
    xw, ss = ops.add_norm_partial(r, slabs.reshape(-1), S, nw)
    _close(r.cpu(), r_ref, atol=1e-2, rtol=1e-2, what="residual")
    _close(ss.sum(1).cpu(), (r_ref.float() ** 2).sum(1), atol=1.0, rtol=1e-3, what="sum of squares")
    y = ops.skinny_linear(xw, ops.pack_skinny(w), rows=M, rownorm=(ss, 1e-5))
    _close(y.cpu(), y_ref, atol=3e-2, rtol=3e-2, what="deferred-norm GEMM")
    ws = ops.skinny_workspace(M, N, 4, DEV)
    ns = ops.skinny_slabs(xw, ops.pack_skinny(w), ws, 4, rows=M, rownorm=(ss, 1e-5))
    _close(ops.reduce_slabs(ws, ns, M, N).cpu(), y_ref, atol=3e-2, rtol=3e-2, what="deferred-norm slabs")


def _paged_prefill_case(cached, new, hq, hkv, D=128, bs=16, spike=False, jumps=None):
    S = len(new)
    tot = [c + n for c, n in zip(cached, new)]
    nblk = [(t + bs - 1) // bs for t in tot]
    NB = sum(nblk) + 3
    kc = torch.randn(NB, hkv, D // 8, bs, 8, device=DEV, dtype=torch.bfloat16)
    vc = torch.randn(NB, hkv, D, bs, device=DEV, dtype=torch.bfloat16)
    perm = torch.randperm(NB, device=DEV).to(torch.int32)
    W = max(nblk) + 5  # wider than needed, as an engine block table is
    bt = torch.zeros(S, W, dtype=torch.int32, device=DEV)
    o = 0
    for i, n in enumerate(nblk):
        bt[i, :n] = perm[o:o + n]
        o += n
    T = sum(new)
    qkv = torch.randn(T, (hq + 2 * hkv) * D, device=DEV, dtype=torch.bfloat16)
    if spike:  # one query row against one key row: the running max jumps late in the sequence
        qkv[T - 1, :D] = 8.0
        qkv[T - 3, (hq) * D:(hq) * D + D] = 8.0
    if jumps:  # q = e_0 on every head, so a score is scale * k[:, 0]; k[:, 0] steps up at given rows
        q3 = qkv.view(T, hq + 2 * hkv, D)
        q3[:, :hq].zero_()
        q3[:, :hq, 0] = 1.0
        q3[:, hq:hq + hkv, 0] = (torch.randn(T, hkv, device=DEV) * 0.5).to(torch.bfloat16)
        level = 0.0
        for row, log2_jump in jumps:  # the running max rises by 2^log2_jump (in exp units) at row
            level += log2_jump * math.log(2) * math.sqrt(D)
            q3[row, hq:hq + hkv, 0] = level
    cu = torch.tensor([0] + list(torch.tensor(new).cumsum(0).tolist()), dtype=torch.int32, device=DEV)
    cs = torch.tensor(cached, dtype=torch.int32, device=DEV)
    pos = torch.cat([torch.arange(c, c + n) for c, n in zip(cached, new)]).to(DEV, torch.int32)
    seq_of = torch.cat([torch.full((n,), i) for i, n in enumerate(new)]).to(DEV)
    slots = (bt[seq_of, (pos // bs).long()] * bs + pos % bs).to(torch.int32)
    ops.rope_and_cache(qkv, pos, torch.zeros(1, D, device=DEV), kc, vc, slots, hq, hkv, D, apply_rope=False)
    return qkv, cu, cs, kc, vc, bt


@pytest.mark.parametrize("order", ["seq", "work"])
@pytest.mark.parametrize("hq,hkv", [(32, 8), (16, 8), (64, 8)])
@pytest.mark.parametrize("cached,new", [([0, 0, 0], [1609, 7, 300]), ([48, 160, 1023], [1, 130, 129]), ([5000], [64])])
def test_flash_prefill_paged_v2_gqa(hq, hkv, cached, new, order):
    """The LDS-DMA paged prefill kernel (v2: tiles staged verbatim from the cache, GQA-shared) ==
    the fp32 reference for G = 2, 4, 8 and cached prefixes, under both q-block orders."""
    D = 128
    qkv, cu, cs, kc, vc, bt = _paged_prefill_case(cached, new, hq, hkv, D)
    qs, st = ops.prefill_qblocks(cu.tolist(), ctx_starts=cached, order=order)
    qb = (torch.tensor(qs, dtype=torch.int32, device=DEV), torch.tensor(st, dtype=torch.int32, device=DEV))
    out = ops.flash_prefill(qkv, cu, hq, hkv, D, 1 / math.sqrt(D), qblocks=qb, paged=(cs, kc, vc, bt))
    exp = ref.paged_prefill(qkv.cpu(), cu.cpu(), cs.cpu(), kc.cpu(), vc.cpu(), bt.cpu(), hq, hkv, D, 1 / math.sqrt(D))
    _close(out.cpu(), exp, atol=2e-2, rtol=2e-2, what=f"paged prefill v2 G={hq // hkv}")


def _attn_rows_fp32(qkv, kc, vc, bt, cached, n_new, rows, hq, hkv, D):
    """fp32 causal attention of the given query rows of ONE sequence (keys = cached prefix + new)."""
    k, v = ref.gather_kv(kc, vc, bt[0], cached + n_new)
    k, v = k.float(), v.float()  # [T, Hkv, D]
    G = hq // hkv
    q = qkv[rows, : hq * D].float().view(len(rows), hkv, G, D)
    s = torch.einsum("rhgd,thd->hgrt", q, k) / math.sqrt(D)
    pos = torch.tensor(rows, device=qkv.device) + cached
    s = s.masked_fill(torch.arange(cached + n_new, device=qkv.device)[None, :] > pos[:, None], float("-inf"))
    o = torch.einsum("hgrt,thd->rhgd", torch.softmax(s, -1), v)
    return o.reshape(len(rows), hq * D)


@pytest.mark.parametrize("cached,new", [(0, 8000), (0, 16000), (3000, 8000)])
def test_flash_prefill_paged_v2_long_prompts(cached, new):
    """the shapes the flash prefill is benchmarked on (8k / 16k new tokens, and a
    chunk after a cached prefix) against fp32 - first, middle and last 256 query rows (the lazy
    reference max sees its longest runs at the end of a long prompt)."""
    hq, hkv, D = 32, 8, 128
    qkv, cu, cs, kc, vc, bt = _paged_prefill_case([cached], [new], hq, hkv, D)
    out = ops.flash_prefill(qkv, cu, hq, hkv, D, 1 / math.sqrt(D), paged=(cs, kc, vc, bt))
    rows = list(range(256)) + list(range(new // 2, new // 2 + 256)) + list(range(new - 256, new))
    exp = _attn_rows_fp32(qkv, kc, vc, bt, cached, new, rows, hq, hkv, D)
    _close(out[rows].float(), exp, atol=2e-2, rtol=2e-2, what=f"paged prefill v2 {cached}+{new}")


@pytest.mark.parametrize("jumps", [[(300, 4), (700, 7), (1300, 6)],           # below the 2^8 threshold
                                   [(200, 7), (230, 7), (900, 10)],          # two in one 64-key tile, then over
                                   [(64, 9), (640, 4), (641, 5), (1500, 8)]])  # exactly at the threshold
def test_flash_prefill_paged_v2_moderate_max_jumps(jumps):
    """The lazy rescale (the reference max moves only on a > 2^8 jump): tile maxima rising by
    2^4 .. 2^10 at chosen rows, every query row against fp32."""
    hq, hkv, D = 32, 8, 128
    new = 1700
    qkv, cu, cs, kc, vc, bt = _paged_prefill_case([37], [new], hq, hkv, D, jumps=jumps)
    out = ops.flash_prefill(qkv, cu, hq, hkv, D, 1 / math.sqrt(D), paged=(cs, kc, vc, bt))
    exp = _attn_rows_fp32(qkv, kc, vc, bt, 37, new, list(range(new)), hq, hkv, D)
    _close(out.float(), exp, atol=2e-2, rtol=2e-2, what=f"paged prefill v2 jumps {jumps}")


def test_flash_prefill_paged_v2_softmax_spike():
    """A late running-max jump (forced by one spiked q/k pair) is rescaled correctly."""
    hq, hkv, D = 32, 8, 128
    qkv, cu, cs, kc, vc, bt = _paged_prefill_case([100], [700], hq, hkv, D, spike=True)
    out = ops.flash_prefill(qkv, cu, hq, hkv, D, 1 / math.sqrt(D), paged=(cs, kc, vc, bt))
    exp = ref.paged_prefill(qkv.cpu(), cu.cpu(), cs.cpu(), kc.cpu(), vc.cpu(), bt.cpu(), hq, hkv, D, 1 / math.sqrt(D))
    _close(out.cpu(), exp, atol=2e-2, rtol=2e-2, what="paged prefill v2 spike")


@pytest.mark.parametrize("hq,hkv", [(32, 8), (8, 8), (24, 8)])
@pytest.mark.parametrize("cached,new", [([0, 32], [40, 7]), ([48, 160, 16], [1, 130, 64]), ([1008], [300])])
def test_flash_prefill_paged(hq, hkv, cached, new):
    """Prefill of new tokens attending a cached prefix in the paged cache == the fp32 reference
    (G = 4 takes the v2 kernel; G = 1 and G = 3 the v1 paged kernel)."""
    D, bs = 128, 16
    S = len(new)
    tot = [c + n for c, n in zip(cached, new)]
    nblk = [(t + bs - 1) // bs for t in tot]
    NB = sum(nblk) + 3
    kc = torch.randn(NB, hkv, D // 8, bs, 8, device=DEV, dtype=torch.bfloat16)
    vc = torch.randn(NB, hkv, D, bs, device=DEV, dtype=torch.bfloat16)
    perm = torch.randperm(NB, device=DEV).to(torch.int32)
    W = max(nblk)
    bt = torch.zeros(S, W, dtype=torch.int32, device=DEV)
    o = 0
    for i, n in enumerate(nblk):
        bt[i, :n] = perm[o:o + n]
        o += n
    T = sum(new)
    qkv = torch.randn(T, (hq + 2 * hkv) * D, device=DEV, dtype=torch.bfloat16)
    cu = torch.tensor([0] + list(torch.tensor(new).cumsum(0).tolist()), dtype=torch.int32, device=DEV)
    cs = torch.tensor(cached, dtype=torch.int32, device=DEV)
    # as in the engine, the new tokens' K/V are in the cache too (rope_and_cache ran first)
    pos = torch.cat([torch.arange(c, c + n) for c, n in zip(cached, new)]).to(DEV, torch.int32)
    seq_of = torch.cat([torch.full((n,), i) for i, n in enumerate(new)]).to(DEV)
    slots = (bt[seq_of, (pos // bs).long()] * bs + pos % bs).to(torch.int32)
    ops.rope_and_cache(qkv, pos, torch.zeros(1, D, device=DEV), kc, vc, slots, hq, hkv, D, apply_rope=False)
    out = ops.flash_prefill(qkv, cu, hq, hkv, D, 1 / math.sqrt(D), paged=(cs, kc, vc, bt))
    exp = ref.paged_prefill(qkv.cpu(), cu.cpu(), cs.cpu(), kc.cpu(), vc.cpu(), bt.cpu(), hq, hkv, D, 1 / math.sqrt(D))
    _close(out.cpu(), exp, atol=2e-2, rtol=2e-2, what="paged prefill")


@pytest.mark.parametrize("M,E", [(1, 4), (24, 8), (64, 2)])
def test_skinny_grouped_moe(M, E):
    """Grouped (grid.z = expert) SwiGLU + routing-weighted down slabs == per-expert fp32 references
    combined with the routing weights (the MoE decode MLP)."""
    K, F, d = 512, 448, 256
    x = torch.randn(M, K, device=DEV, dtype=torch.bfloat16)
    w13 = (torch.randn(E, 2 * F, K, device=DEV) * 0.05).to(torch.bfloat16)
    w2 = (torch.randn(E, d, F, device=DEV) * 0.05).to(torch.bfloat16)
    wd = torch.rand(M, E, device=DEV) * (torch.rand(M, E, device=DEV) > 0.5)
    w13p = torch.stack([ops.pack_skinny(ops.interleave_gate_up(w)) for w in w13])
    w2p = torch.stack([ops.pack_skinny(w) for w in w2])
    act = ops.skinny_grouped_swiglu(ops.pack_activation(x), w13p, rows=M)
    ws = torch.empty(E * M * d, device=DEV, dtype=torch.float32)
    ns = ops.skinny_grouped_slabs(act, w2p, ws, M, wd, splits=1)
    assert ns == E
    out = ws[: E * M * d].view(E, M, d).sum(0)
    ref_out = torch.zeros(M, d)
    for e in range(E):
        gu = torch.nn.functional.linear(x.cpu().float(), w13[e].cpu().float()).to(torch.bfloat16)
        a = ref.silu_mul(gu)
        _close(ops.unpack_skinny(act[e])[:M].cpu(), a, atol=3e-2, rtol=2e-2, what=f"expert {e} act")
        ref_out += torch.nn.functional.linear(a.float(), w2[e].cpu().float()) * wd[:, e:e + 1].cpu()
    _close(out.cpu(), ref_out, atol=6e-2, rtol=3e-2, what="weighted combine")


@pytest.mark.parametrize("n", [1, 37, 64])
def test_resolve_ids(n):
    ids = torch.randint(0, 1000, (n,), dtype=torch.int32, device=DEV)
    prev = torch.randint(0, 1000, (64,), dtype=torch.int32, device=DEV)
    src = torch.randint(-1, 64, (n,), dtype=torch.int32, device=DEV)
    y = ops.resolve_ids(ids, src, prev)
    r = torch.where(src.cpu() >= 0, prev.cpu()[src.cpu().clamp(min=0).long()], ids.cpu())
    assert torch.equal(y.cpu(), r)


@pytest.mark.parametrize("d", [128, 64])
def test_rope_and_cache_prefill_block_runs(d):
    """Prefill layout: sequences' new tokens are consecutive slots inside their blocks, chunks start
    mid-block and sequences at arbitrary rows - the block-run cache writer must match the reference
    (full 16-token runs, ragged starts / ends, runs crossing the 16-row windows, padding rows)."""
    hq, hkv, bs = 8, 4, 16
    starts, lens = [0, 5, 16, 37, 3], [40, 27, 16, 1, 70]  # ctx_start (first position), new tokens
    nb = 64
    perm = torch.randperm(nb)
    ids_slots, pos_l, used = [], [], 0
    for c, n in zip(starts, lens):
        nblk = (c + n + bs - 1) // bs
        bt = perm[used:used + nblk]
        used += nblk
        p = torch.arange(c, c + n)
        pos_l.append(p)
        ids_slots.append(bt[p // bs] * bs + p % bs)
    slots = torch.cat(ids_slots).to(torch.int32)
    slots[7] = -1  # a padding row inside a run
    pos = torch.cat(pos_l).to(torch.int32)
    T = slots.numel()
    qkv = torch.randn(T, (hq + 2 * hkv) * d, device=DEV, dtype=torch.bfloat16)
    cs = ref.rope_cos_sin(4096, d, 500000.0, device=DEV)
    kc, vc = _make_cache(nb, hkv, d)
    kc0, vc0 = kc.clone().cpu(), vc.clone().cpu()
    q2 = qkv.clone().cpu()
    ops.rope_and_cache(qkv, pos.to(DEV), cs, kc, vc, slots.to(DEV), hq, hkv, d)
    ref.rope_and_cache(q2, pos, cs.cpu(), kc0, vc0, slots, hq, hkv, d)
    _close(qkv, q2.to(DEV), atol=2e-2, rtol=1e-2, what="rope qkv")
    _close(kc, kc0.to(DEV), atol=2e-2, rtol=1e-2, what="k_cache")
    assert torch.equal(vc.cpu(), vc0), "v_cache"
