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


ALGOS = [0, 1, 2]  # 4-wave kernel: 0 one barrier per k-tile, 1 two; 2 the 8-wave ping-pong kernel (gemm_pp.hip)
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
