"""The 256 x 256 MFMA prefill GEMM (ops/csrc/gemm_tile.hip): dense and expert-grouped, plain and
SwiGLU epilogues, against plain PyTorch fp32 references of the same op."""
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


ALGOS = [0, 1]  # the 4-wave kernel: 0 one barrier per k-tile, 1 two
DENSE_ALGOS = ALGOS


@pytest.mark.parametrize("algo", DENSE_ALGOS)
@pytest.mark.parametrize("M,N,K", [(1, 256, 64), (255, 512, 128), (300, 256, 192), (1000, 1536, 1024),
                                   (2048, 768, 4096), (513, 512, 14336 // 4), (4096, 1024, 640)])
def test_gemm_tile_dense(M, N, K, algo):
    x = torch.randn(M, K, device=DEV, dtype=torch.bfloat16)
    w = (torch.randn(N, K, device=DEV) * 0.05).to(torch.bfloat16)
    y = ops.gemm_tile(x, w, algo=algo)
    _close(y.cpu(), F_.linear(x.cpu().float(), w.cpu().float()), atol=3e-2, rtol=2e-2, what=f"dense {M}x{N}x{K}")


@pytest.mark.parametrize("M,N", [(77, 400), (600, 16), (257, 1296)])
def test_gemm_tile_w4_n_tail(M, N):
    """The 4-wave kernel takes any N % 16 == 0 (partial last n-tile: clamped DMA rows, masked stores)."""
    K = 320
    x = torch.randn(M, K, device=DEV, dtype=torch.bfloat16)
    w = (torch.randn(N, K, device=DEV) * 0.05).to(torch.bfloat16)
    for algo in ALGOS:
        y = ops.gemm_tile(x, w, algo=algo)
        _close(y.cpu(), F_.linear(x.cpu().float(), w.cpu().float()), atol=3e-2, rtol=2e-2, what=f"tail {M}x{N}")


def test_gemm_tile_w4_asymmetric_identity():
    """A = I with an asymmetric B: a transposed C-write or a swapped fragment map cannot pass."""
    K = 256
    x = torch.zeros(256, K, device=DEV, dtype=torch.bfloat16)
    x[:, :] = torch.eye(256, K, device=DEV, dtype=torch.bfloat16)
    n = torch.arange(512, device=DEV).float()[:, None]
    k = torch.arange(K, device=DEV).float()[None, :]
    w = ((n * 3 + k * 7) % 61 - 30).to(torch.bfloat16)  # small integers: exact in bf16
    for algo in ALGOS:
        y = ops.gemm_tile(x, w, algo=algo)
        assert torch.equal(y.float().cpu(), w.float().t().cpu()[:256])


@pytest.mark.parametrize("algo", DENSE_ALGOS)
@pytest.mark.parametrize("M", [7, 700])
def test_gemm_tile_swiglu(M, algo):
    K, F = 512, 768
    x = torch.randn(M, K, device=DEV, dtype=torch.bfloat16)
    w13 = (torch.randn(2 * F, K, device=DEV) * 0.05).to(torch.bfloat16)
    y = ops.gemm_tile(x, ops.interleave_gate_up(w13).contiguous(), swiglu=True, algo=algo)
    r = ref.silu_mul(F_.linear(x.cpu().float(), w13.cpu().float()).to(torch.bfloat16))
    _close(y.cpu(), r, atol=3e-2, rtol=2e-2, what="swiglu")


@pytest.mark.parametrize("algo", ALGOS)
@pytest.mark.parametrize("counts", [[300, 0, 129, 1], [256, 512, 5, 700, 0, 0, 33, 64], [1]])
@pytest.mark.parametrize("swiglu", [False, True])
def test_gemm_tile_grouped(counts, swiglu, algo):
    E, K, N = len(counts), 512, 512
    rows = sum(counts)
    x = torch.randn(rows, K, device=DEV, dtype=torch.bfloat16)
    w = (torch.randn(E, N, K, device=DEV) * 0.05).to(torch.bfloat16)
    if swiglu:
        w = torch.stack([ops.interleave_gate_up(we) for we in w]).contiguous()
    off = torch.tensor([0] + torch.tensor(counts).cumsum(0).tolist(), dtype=torch.int32, device=DEV)
    y = ops.gemm_tile(x, w, off, swiglu=swiglu, algo=algo)
    o = 0
    for e, n in enumerate(counts):
        if n:
            r = F_.linear(x[o:o + n].cpu().float(), w[e].cpu().float()).to(torch.bfloat16)
            if swiglu:
                r = ref.silu_mul(r, interleaved=True)
            _close(y[o:o + n].cpu(), r, atol=3e-2, rtol=2e-2, what=f"expert {e}")
        o += n


def test_gemm_tile_grouped_local_slice():
    """A rank's slice of the offsets: other experts' rows stay as allocated (zero)."""
    counts = [200, 150, 90, 310]
    E, K, N = 4, 256, 256
    x = torch.randn(sum(counts), K, device=DEV, dtype=torch.bfloat16)
    w = (torch.randn(E, N, K, device=DEV) * 0.05).to(torch.bfloat16)
    off = torch.tensor([0] + torch.tensor(counts).cumsum(0).tolist(), dtype=torch.int32, device=DEV)
    y = ops.gemm_tile(x, w[1:3].contiguous(), off[1:4])
    assert int(y[:200].abs().sum()) == 0 and int(y[440:].abs().sum()) == 0
    for e, (a, b) in ((1, (200, 350)), (2, (350, 440))):
        _close(y[a:b].cpu(), F_.linear(x[a:b].cpu().float(), w[e].cpu().float()), atol=3e-2, rtol=2e-2,
               what=f"local expert {e}")


def test_gemm_tile_in_graph_matches_eager():
    x = torch.randn(600, 1024, device=DEV, dtype=torch.bfloat16)
    w = (torch.randn(1024, 1024, device=DEV) * 0.03).to(torch.bfloat16)
    y0 = ops.gemm_tile(x, w)
    out = torch.empty_like(y0)
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    with torch.cuda.stream(s), torch.cuda.graph(g, stream=s):
        ops.gemm_tile(x, w, out=out)
    g.replay()
    torch.cuda.synchronize()
    assert torch.equal(out, y0)


@pytest.mark.parametrize("algo", ALGOS)
@pytest.mark.parametrize("M,N,K", [(300, 256, 192), (1000, 1536, 1024), (257, 1296, 640), (2048, 768, 4096)])
def test_gemm_tile_packed_weights_bit_identical(M, N, K, algo):
    """W in the decode GEMMs' fragment-packed layout (pack_skinny) gives the same bits as W
    row-major: only the DMA source / LDS image of W change, not the MFMA operands or their order -
    plain, SwiGLU, grouped, RoPE + row scale and the residual epilogue."""
    x = torch.randn(M, K, device=DEV, dtype=torch.bfloat16)
    w = (torch.randn(N, K, device=DEV) * 0.05).to(torch.bfloat16)
    assert torch.equal(ops.gemm_tile(x, ops.pack_skinny(w), algo=algo), ops.gemm_tile(x, w, algo=algo))
    if N % 256 == 0:
        wi = ops.interleave_gate_up(w).contiguous()
        assert torch.equal(ops.gemm_tile(x, ops.pack_skinny(wi), swiglu=True, algo=algo),
                           ops.gemm_tile(x, wi, swiglu=True, algo=algo))
    counts = [M // 3, 0, M - M // 3]
    off = torch.tensor([0] + torch.tensor(counts).cumsum(0).tolist(), dtype=torch.int32, device=DEV)
    we = torch.stack([w, w.flip(0), w * 0.5]).contiguous()
    wep = torch.stack([ops.pack_skinny(e) for e in we]).contiguous()
    assert torch.equal(ops.gemm_tile(x, wep, off, algo=algo), ops.gemm_tile(x, we, off, algo=algo))
    if algo == 1 and K >= 192 and K % 128 == 0 and N % 128 == 0:
        pos = torch.arange(M, device=DEV, dtype=torch.int32)
        cs = ref.rope_cos_sin(4096, 128, 500000.0).to(DEV).float().contiguous()
        ss = (torch.rand(M, K // 128, device=DEV) * 64 + 16).contiguous()
        kw = dict(algo=1, rope=(pos, cs, N // 128), rowscale=(ss, 1e-5))
        assert torch.equal(ops.gemm_tile(x, ops.pack_skinny(w), **kw), ops.gemm_tile(x, w, **kw))
        resid = torch.randn(M, N, device=DEV, dtype=torch.bfloat16)
        nw = (torch.rand(N, device=DEV) + 0.5).to(torch.bfloat16)
        r1, r2 = resid.clone(), resid.clone()
        h1, s1 = ops.gemm_tile_resid(x, ops.pack_skinny(w), r1, nw)
        h2, s2 = ops.gemm_tile_resid(x, w, r2, nw)
        assert torch.equal(r1, r2) and torch.equal(h1, h2) and torch.equal(s1, s2)


@pytest.mark.parametrize("M", [7, 700, 1500])
@pytest.mark.parametrize("rowscale", [False, True])
def test_gemm_tile_swiglu8_matches_fp32_and_decode_layout(M, rowscale):
    """SwiGLU over the decode GEMMs' gate/up copy (interleave_gate_up8, fragment-packed): the
    features silu(gate) * up against fp32, row-major vs packed bit for bit, dense and grouped -
    the one weight copy prefill and decode share."""
    K, F = 512, 768
    x = torch.randn(M, K, device=DEV, dtype=torch.bfloat16)
    w13 = (torch.randn(2 * F, K, device=DEV) * 0.05).to(torch.bfloat16)
    w8 = ops.interleave_gate_up8(w13).contiguous()
    kw = {}
    xs = x.cpu().float()
    if rowscale:
        ss = (torch.rand(M, K // 128, device=DEV) * 64 + 16).contiguous()
        kw = dict(algo=1, rowscale=(ss, 1e-5))
        xs = xs * torch.rsqrt(ss.cpu().sum(1, keepdim=True) / K + 1e-5)
    y = ops.gemm_tile(x, ops.pack_skinny(w8), swiglu=8, **kw)
    assert torch.equal(y, ops.gemm_tile(x, w8, swiglu=8, **kw))
    gu = F_.linear(xs, w13.cpu().float()).to(torch.bfloat16).float()
    r = F_.silu(gu[:, :F]) * gu[:, F:]
    _close(y.cpu(), r, atol=3e-2, rtol=2e-2, what="swiglu8")
    if not rowscale:
        counts = [M // 2, M - M // 2]
        off = torch.tensor([0, counts[0], M], dtype=torch.int32, device=DEV)
        we = torch.stack([ops.pack_skinny(w8), ops.pack_skinny(w8.flip(1).contiguous())]).contiguous()
        yg = ops.gemm_tile(x, we, off, swiglu=8)
        assert torch.equal(yg[: counts[0]], y[: counts[0]])
