"""The row-major skinny GEMM (gemm_skinny_rm_kernel: W streamed as whole 128-B lines by LDS-DMA
from the plain [N, K] weight, the single resident copy) against the fp32 reference, for every
epilogue the decode path uses, and bit-for-bit against the fragment-packed kernel it replaces."""
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


def _w(N, K, s=0.05):
    return (torch.randn(N, K, device=DEV, dtype=torch.bfloat16) * s).to(torch.bfloat16)


@pytest.mark.parametrize("M,N,K,splits", [(1, 256, 512, 1), (16, 512, 1024, 2), (33, 384, 4096, 4),
                                          (64, 6144, 4096, 2), (64, 4096, 4096, 4), (5, 192, 1344, 3)])
def test_rm_slabs_and_bf16(M, N, K, splits):
    a = torch.randn(M, K, device=DEV, dtype=torch.bfloat16)
    w = _w(N, K)
    ap = ops.pack_activation(a)
    y_ref = F_.linear(a.cpu().float(), w.cpu().float())
    ws = ops.skinny_workspace(M, N, max(splits, 1), DEV)
    ns = ops.skinny_slabs(ap, w, ws, splits, rows=M)
    y = ops.reduce_slabs(ws, ns, M, N)
    _close(y.cpu(), y_ref, atol=3e-2, rtol=2e-2, what=f"rm slabs M{M} N{N} K{K} s{splits}")
    ws2 = ops.skinny_workspace(M, N, max(splits, 1), DEV)
    ns2 = ops.skinny_slabs(ap, ops.pack_skinny(w), ws2, splits, rows=M)
    assert ns2 == ns
    # same fragments, same k order inside each wave: the packed kernel's partial sums match closely
    _close(ws[: ns * M * N].cpu(), ws2[: ns * M * N].cpu(), atol=2e-3, rtol=1e-3, what="rm vs packed slabs")
    y1 = ops.skinny_linear(ap, w, rows=M)
    _close(y1.cpu(), y_ref, atol=3e-2, rtol=2e-2, what="rm bf16 epilogue")


@pytest.mark.parametrize("M", [1, 20, 64])
def test_rm_swiglu_packed_feeds_down(M):
    K, F, d = 1024, 448, 512
    x = torch.randn(M, K, device=DEV, dtype=torch.bfloat16)
    w13 = _w(2 * F, K)
    w2 = _w(d, F)
    gu = F_.linear(x.cpu().float(), w13.cpu().float()).to(torch.bfloat16)
    act_ref = ref.silu_mul(gu)
    actp = ops.skinny_swiglu(ops.pack_activation(x), ops.interleave_gate_up(w13).contiguous(), rows=M,
                             packed_out=True)
    _close(ops.unpack_skinny(actp)[:M].cpu(), act_ref, atol=3e-2, rtol=2e-2, what="rm swiglu packed")
    act = ops.skinny_swiglu(ops.pack_activation(x), ops.interleave_gate_up(w13).contiguous(), rows=M)
    _close(act.cpu(), act_ref, atol=3e-2, rtol=2e-2, what="rm swiglu row-major out")
    y = ops.skinny_linear(actp, w2, rows=M)
    _close(y.cpu(), F_.linear(act_ref.float(), w2.cpu().float()), atol=4e-2, rtol=3e-2, what="rm down")


@pytest.mark.parametrize("M", [3, 64])
def test_rm_deferred_rmsnorm(M):
    K, N = 4096, 1024
    x = torch.randn(M, K, device=DEV, dtype=torch.bfloat16)
    nw = (torch.rand(K, device=DEV) + 0.5).to(torch.bfloat16)
    w = _w(N, K, 0.02)
    xw, ss = ops.add_norm_partial(x.clone(), None, 0, nw)
    y = ops.skinny_linear(xw, w, rows=M, rownorm=(ss, 1e-5))
    y_ref = F_.linear(ref.rms_norm(x.cpu(), nw.cpu(), 1e-5).float(), w.cpu().float())
    _close(y.cpu(), y_ref, atol=3e-2, rtol=3e-2, what="rm deferred norm")


@pytest.mark.parametrize("M,E", [(1, 4), (64, 2), (100, 2), (128, 4)])
def test_rm_grouped_moe(M, E):
    """Grouped gate/up + SwiGLU and down over every local expert; 65..128 rows take the 8-m-tile
    2-wave form (the EP all-to-all decode's received rows in one launch)."""
    K, F, d = 512, 448, 256
    x = torch.randn(M, K, device=DEV, dtype=torch.bfloat16)
    w13 = (torch.randn(E, 2 * F, K, device=DEV) * 0.05).to(torch.bfloat16)
    w2 = (torch.randn(E, d, F, device=DEV) * 0.05).to(torch.bfloat16)
    wd = torch.rand(M, E, device=DEV)
    w13i = torch.stack([ops.interleave_gate_up(w) for w in w13]).contiguous()
    act = ops.skinny_grouped_swiglu(ops.pack_activation(x), w13i, rows=M)
    ws = torch.empty(E * M * d, device=DEV, dtype=torch.float32)
    ns = ops.skinny_grouped_slabs(act, w2, ws, M, wd, splits=1)
    out = ws[: ns * M * d].view(ns, M, d).sum(0)
    ref_out = torch.zeros(M, d)
    for e in range(E):
        a = ref.silu_mul(F_.linear(x.cpu().float(), w13[e].cpu().float()).to(torch.bfloat16))
        ref_out += F_.linear(a.float(), w2[e].cpu().float()) * wd[:, e:e + 1].cpu()
    _close(out.cpu(), ref_out, atol=6e-2, rtol=3e-2, what="rm grouped moe")


@pytest.mark.parametrize("M", [40, 64])
def test_rm_deferred_rmsnorm_two_wave_grids(M):
    """Grids of more than one round of 4-wave workgroups run 2-wave workgroups (gate_up at
    F = 14336: 448 tiles; the LM head: 2004): every row's 1/rms must reach the epilogue, not only
    the first 32 rows' (4 threads per row cover 32 rows per pass of a 128-thread workgroup)."""
    K, F = 4096, 14336
    x = torch.randn(M, K, device=DEV, dtype=torch.bfloat16)
    nw = (torch.rand(K, device=DEV) + 0.5).to(torch.bfloat16)
    xn = ref.rms_norm(x.cpu(), nw.cpu(), 1e-5).to(DEV).float()
    xw, ss = ops.add_norm_partial(x.clone(), None, 0, nw)
    w13 = _w(2 * F, K, 0.02)
    act = ops.skinny_swiglu(xw, ops.interleave_gate_up(w13).contiguous(), rows=M, rownorm=(ss, 1e-5))
    act_ref = ref.silu_mul((xn @ w13.float().t()).to(torch.bfloat16).cpu())
    _rows_close(act.cpu(), act_ref, f"rm swiglu deferred norm, 448 tiles, M{M}")
    w = _w(32768, K, 0.02)  # 512 tiles: the bf16 epilogue (LM-head form)
    y = ops.skinny_linear(xw, w, rows=M, rownorm=(ss, 1e-5))
    _rows_close(y.cpu(), (xn @ w.float().t()).cpu(), f"rm linear deferred norm, M{M}")


def _rows_close(a, b, what, tol=1e-2):
    """Per-row relative error (bf16 double rounding of the normed input moves single elements by a
    few ulps; a missing 1/rms moves the whole row)."""
    e = ((a.float() - b.float()).norm(dim=1) / b.float().norm(dim=1).clamp_min(1e-6))
    bad = (e > tol).nonzero().flatten().tolist()
    assert not bad, f"{what}: rows {bad[:8]} off by {e.max().item():.3g} (relative)"
