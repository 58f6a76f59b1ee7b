"""The 8-wave ping-pong prefill GEMM (ops/csrc/gemm_pp.hip, gemm_tile algo 2) against the 4-wave
kernel (algo 1) it replaces: the same MFMA accumulation order per output element and the same
epilogue arithmetic, so every output must be BIT-identical - plain, SwiGLU, RoPE, residual-add /
next-norm, the deferred-norm row scale, and expert-grouped launches, at Llama-3-8B prefill shapes
with ragged row / column tails.  (Both are checked against fp32 references in
test_gemm_tile_gpu.py / test_tile_real_shapes_gpu.py.)"""
import pytest
import torch

from k8s_llm_monitor_amd import ops
from k8s_llm_monitor_amd.ops import reference as ref

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.fixture(autouse=True, scope="module")
def _native_loaded():
    ops.native()


def _rand(*shape, s=1.0, seed=0):
    g = torch.Generator(device=DEV).manual_seed(seed)
    return (torch.randn(*shape, device=DEV, generator=g) * s).to(torch.bfloat16)


@pytest.mark.parametrize("M,N,K", [(1024, 4096, 4096), (1609, 6144, 4096), (300, 4096, 14336), (777, 4208, 512),
                                   (256, 272, 128)])
def test_pp_dense_bitwise(M, N, K):
    x, w = _rand(M, K, seed=1), _rand(N, K, s=0.02, seed=2)
    a = ops.gemm_tile(x, w, algo=1)
    b = ops.gemm_tile(x, w, algo=2)
    assert torch.equal(a, b)
    ref_ = x.float() @ w.float().t()
    assert (b.float() - ref_).abs().max().item() <= 2e-2 * ref_.abs().max().item()


@pytest.mark.parametrize("M", [1024, 1609, 4096])
def test_pp_swiglu_bitwise(M):
    d, F = 4096, 14336
    x, w13 = _rand(M, d, seed=3), _rand(2 * F, d, s=0.02, seed=4)
    wi = ops.interleave_gate_up(w13).contiguous()
    assert torch.equal(ops.gemm_tile(x, wi, swiglu=True, algo=1), ops.gemm_tile(x, wi, swiglu=True, algo=2))


@pytest.mark.parametrize("M", [1024, 1609])
def test_pp_rope_and_rowscale_bitwise(M):
    d, F, Hq, Hk = 4096, 14336, 32, 8
    h = _rand(M, d, s=3.0, seed=5)
    nw = (torch.rand(d, device=DEV) + 0.5).to(torch.bfloat16)
    hw = (h.float() * nw.float()).to(torch.bfloat16)
    ss = (h.float() ** 2).view(M, d // 128, 128).sum(2).contiguous()
    wq = _rand(6144, d, s=0.02, seed=6)
    cs = ref.rope_cos_sin(4096, 128, 500000.0).to(DEV).float().contiguous()
    pos = (torch.arange(M, device=DEV) % 4096).to(torch.int32)
    for rs in (None, (ss, 1e-5)):
        a = ops.gemm_tile(hw, wq, algo=1, rope=(pos, cs, Hq + Hk), rowscale=rs)
        b = ops.gemm_tile(hw, wq, algo=2, rope=(pos, cs, Hq + Hk), rowscale=rs)
        assert torch.equal(a, b), f"rope rowscale={rs is not None}"
    wi = ops.interleave_gate_up(_rand(2 * F, d, s=0.02, seed=7)).contiguous()
    a = ops.gemm_tile(hw, wi, swiglu=True, algo=1, rowscale=(ss, 1e-5))
    b = ops.gemm_tile(hw, wi, swiglu=True, algo=2, rowscale=(ss, 1e-5))
    assert torch.equal(a, b)


@pytest.mark.parametrize("M,K", [(1024, 4096), (1609, 14336)])
def test_pp_resid_bitwise(M, K, monkeypatch):
    d = 4096
    x, w = _rand(M, K, seed=8), _rand(d, K, s=0.02, seed=9)
    res0 = _rand(M, d, seed=10)
    nw = (torch.rand(d, device=DEV) + 0.5).to(torch.bfloat16)
    outs = {}
    for algo in (1, 2):
        monkeypatch.setattr(ops, "TILE_ALGO", algo)
        r = res0.clone()
        hw, ss = ops.gemm_tile_resid(x, w, r, nw)
        outs[algo] = (r, hw, ss)
    for u, v in zip(outs[1], outs[2]):
        assert torch.equal(u, v)


@pytest.mark.parametrize("swiglu", [False, True])
def test_pp_grouped_bitwise(swiglu):
    E, d, F = 8, 4096, 1024
    counts = [700, 0, 33, 256, 1, 900, 0, 130]
    T = sum(counts)
    x = _rand(T, d, seed=11)
    w = _rand(E, 2 * F if swiglu else d, d, s=0.02, seed=12)
    if swiglu:
        w = torch.stack([ops.interleave_gate_up(e) for e in w]).contiguous()
    off = torch.tensor([0] + list(torch.tensor(counts).cumsum(0)), dtype=torch.int32, device=DEV)
    a = ops.gemm_tile(x, w, off, swiglu=swiglu, algo=1)
    b = ops.gemm_tile(x, w, off, swiglu=swiglu, algo=2)
    assert torch.equal(a, b)
