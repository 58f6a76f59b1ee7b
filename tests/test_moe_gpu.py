"""MoE on the GPU: the grouped expert GEMM (ops/csrc/moe_gemm.hip, one launch over every local
expert, device-side offsets) against per-expert fp32 references, and the Mixtral prefill layer
with the grouped path against the per-expert hipBLASLt loop."""
import pytest
import torch

from k8s_llm_monitor_amd import ops
from k8s_llm_monitor_amd.ops import reference as ref

pytestmark = pytest.mark.gpu
DEV = "cuda"
F_ = torch.nn.functional


@pytest.fixture(autouse=True, scope="module")
def _native_loaded():
    ops.native()
    torch.manual_seed(0)


def _close(a, b, atol, rtol=0.0, what=""):
    err = (a.float() - b.float()).abs()
    tol = atol + rtol * b.float().abs()
    bad = (err > tol).sum().item()
    assert bad == 0, f"{what}: {bad} elements out of tolerance, max err {err.max().item():.4g}"


@pytest.mark.parametrize("counts", [[300, 0, 129, 1], [128, 128, 5, 700, 0, 0, 33, 64], [1]])
@pytest.mark.parametrize("swiglu", [False, True])
def test_moe_grouped_gemm(counts, swiglu):
    E, K, N = len(counts), 512, 384
    rows = sum(counts)
    x = torch.randn(rows, K, device=DEV, dtype=torch.bfloat16)
    w = (torch.randn(E, N, K, device=DEV) * 0.05).to(torch.bfloat16)
    if swiglu:
        w = torch.stack([ops.interleave_gate_up(we) for we in w]).contiguous()
    off = torch.tensor([0] + torch.tensor(counts).cumsum(0).tolist(), dtype=torch.int32, device=DEV)
    y = ops.moe_grouped_gemm(x, w, off, swiglu=swiglu)
    o = 0
    for e, n in enumerate(counts):
        if n == 0:
            continue
        r = F_.linear(x[o:o + n].cpu().float(), w[e].cpu().float()).to(torch.bfloat16)
        if swiglu:
            r = ref.silu_mul(r, interleaved=True)
        _close(y[o:o + n].cpu(), r, atol=3e-2, rtol=2e-2, what=f"expert {e}")
        o += n


def test_moe_grouped_gemm_local_expert_slice():
    """A rank's slice of the offsets (its experts only): other experts' rows stay zero."""
    counts = [200, 150, 90, 310]
    E, K, N = 4, 256, 256
    rows = sum(counts)
    x = torch.randn(rows, K, device=DEV, dtype=torch.bfloat16)
    w = (torch.randn(E, N, K, device=DEV) * 0.05).to(torch.bfloat16)
    off = torch.tensor([0] + torch.tensor(counts).cumsum(0).tolist(), dtype=torch.int32, device=DEV)
    y = ops.moe_grouped_gemm(x, w[1:3].contiguous(), off[1:4])
    assert int(y[:200].abs().sum()) == 0 and int(y[440:].abs().sum()) == 0
    for e, (a, b) in ((1, (200, 350)), (2, (350, 440))):
        _close(y[a:b].cpu(), F_.linear(x[a:b].cpu().float(), w[e].cpu().float()), atol=3e-2, rtol=2e-2,
               what=f"local expert {e}")


def test_mixtral_prefill_grouped_matches_loop(monkeypatch):
    """A Mixtral prefill forward with the grouped expert GEMMs == the per-expert hipBLASLt loop."""
    from k8s_llm_monitor_amd.models.config import get_config
    from k8s_llm_monitor_amd.models.llama import AttnMeta, CausalLM

    cfg = get_config("mixtral-tiny-d128")
    m = CausalLM(cfg, device=DEV, seed=3)
    T = 300
    ids = torch.randint(0, cfg.vocab_size, (T,), device=DEV, dtype=torch.int32)
    cu = torch.tensor([0, 180, T], dtype=torch.int32, device=DEV)
    meta = AttnMeta(is_prefill=True, positions=torch.cat([torch.arange(180), torch.arange(T - 180)]).to(DEV, torch.int32),
                    slot_mapping=torch.full((T,), -1, dtype=torch.int32, device=DEV), cu_seqlens=cu)
    m._moe_grouped = True
    a = m.forward(ids, meta)
    m._moe_grouped = False
    b = m.forward(ids, meta)
    _close(a.float().cpu(), b.float().cpu(), atol=5e-2, rtol=5e-2, what="grouped vs loop logits")
    assert torch.equal(a.argmax(-1), b.argmax(-1)) or (a.argmax(-1) == b.argmax(-1)).float().mean() > 0.98


@pytest.mark.parametrize("T", [96, 128])
def test_moe_decode_beyond_skinny_rows_grouped_in_graph(T):
    """Decode MoE with more rows than the skinny kernels take (max_num_seqs > 64): the routed,
    grouped path (moe_align + one grouped GEMM per projection, device offsets) matches an fp32
    per-token reference of the same weights and replays from a hipGraph (no host sync inside)."""
    from k8s_llm_monitor_amd.models import AttnMeta, CausalLM, get_config

    cfg = get_config("mixtral-tiny").replace(d_model=512, ffn_dim=1024)
    gm = CausalLM(cfg, device=DEV, seed=21)
    L = gm.layers[0]
    x = (torch.randn(T, cfg.d_model, device=DEV) * 0.5).to(torch.bfloat16)
    meta = AttnMeta(is_prefill=False, positions=torch.zeros(T, dtype=torch.int32, device=DEV),
                    slot_mapping=torch.full((T,), -1, dtype=torch.int32, device=DEV))
    y = gm._moe(L, x, meta).float()
    # fp32 reference: softmax top-k routing, renormalised, then the selected experts per token
    xf = x.float()
    probs = torch.softmax(xf @ L["router"].float().t(), -1)
    tw, ti = probs.topk(cfg.top_k_experts, -1)
    tw = tw / tw.sum(-1, keepdim=True)
    F = cfg.ffn_dim
    r = torch.zeros_like(xf)
    w13s, w2s = gm.canonical(L, "w13"), gm.canonical(L, "w2")  # [gate; up] whatever the resident layout
    for e in range(cfg.n_experts):
        gu = xf @ w13s[e].float().t()
        h = (F_.silu(gu[:, :F]) * gu[:, F:]) @ w2s[e].float().t()
        r += h * (tw * (ti == e)).sum(-1, keepdim=True)
    _close(y, r, atol=5e-2, rtol=5e-2, what=f"decode moe T{T}")
    xs = x.clone()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        gm._moe(L, xs, meta)
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        yg = gm._moe(L, xs, meta)
    g.replay()
    torch.cuda.synchronize()
    assert torch.equal(yg.float(), y)


@pytest.mark.parametrize("T", [1, 64, 300])
@pytest.mark.parametrize("E,K", [(8, 2), (16, 4)])
def test_moe_router_matches_linear_route_scatter(T, E, K):
    """The one-launch MoE router (moe_router_kernel) = bf16 F.linear -> fp32 -> moe_route -> dense
    per-expert weight rows: same experts, same weights (fp32 tolerance)."""
    d = 4096
    # small integers x 2^-7: every partial sum is exact in fp32, so both accumulation orders give
    # the same logits (no bf16-rounding flips of a near-tie between the two paths)
    g = torch.Generator(device="cuda").manual_seed(T * 31 + E)
    x = torch.randint(-2, 3, (T, d), device="cuda", generator=g).to(torch.bfloat16)
    wr = (torch.randint(-8, 9, (E, d), device="cuda", generator=g).float() / 128).to(torch.bfloat16)
    ids, w, wd = ops.moe_router(x, wr, K, True)
    lg = torch.nn.functional.linear(x.float(), wr.float()).to(torch.bfloat16).float()
    rids, rw = ops.moe_route(lg, K, True)
    assert torch.equal(ids, rids)
    torch.testing.assert_close(w, rw, rtol=1e-5, atol=1e-6)
    ref_wd = torch.zeros(T, E, device="cuda").scatter_(1, rids.long(), rw)
    torch.testing.assert_close(wd, ref_wd, rtol=1e-5, atol=1e-6)


def test_moe_router_nan_rows_pick_valid_experts():
    """A row whose router logits are NaN (a poisoned activation) must still yield K distinct, valid
    expert ids and write only inside its own dense weight row (best = -1 indexed
    wd[t*E - 1], the neighbouring row)."""
    T, E, K, d = 4, 8, 2, 4096
    g = torch.Generator(device="cuda").manual_seed(7)
    x = torch.randn(T, d, device="cuda", generator=g).to(torch.bfloat16)
    x[1, 5] = float("nan")
    wr = (torch.randn(E, d, device="cuda", generator=g) * 0.02).to(torch.bfloat16)
    ids, w, wd = ops.moe_router(x, wr, K, True)
    ids = ids.cpu()
    assert ((ids >= 0) & (ids < E)).all()
    assert all(len(set(r.tolist())) == K for r in ids)
    # the healthy rows are untouched by the poisoned one: same result as routing them alone
    keep = torch.tensor([0, 2, 3], device="cuda")
    ids2, w2, wd2 = ops.moe_router(x[keep].contiguous(), wr, K, True)
    assert torch.equal(ids[keep.cpu()], ids2.cpu())
    torch.testing.assert_close(wd[keep], wd2)
