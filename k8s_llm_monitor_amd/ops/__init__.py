"""Fused operators.  GPU tensors run the gfx950 HIP kernels of ``_k8sllm_ops`` (built in-tree by
``python -m k8s_llm_monitor_amd.ops.build``); CPU tensors run the fp32 references of
:mod:`.reference` (attention: the batched SDPA forms of :mod:`.cpu_attn`, same math).  A GPU tensor never silently falls back: if the extension is missing on a
GPU box the call raises, so tests and benchmarks always exercise the native kernels.
"""
from __future__ import annotations

import importlib
import math
from typing import Optional

import torch

from . import cpu_attn
from . import reference as ref

_EXT = None
_EXT_ERR: Optional[BaseException] = None


def native():
    """The compiled extension module (raises with the build hint if unavailable)."""
    global _EXT, _EXT_ERR
    if _EXT is None and _EXT_ERR is None:
        try:
            _EXT = importlib.import_module("k8s_llm_monitor_amd.ops._k8sllm_ops")
        except BaseException as e:  # noqa: BLE001 - remember why, re-raise on GPU use
            _EXT_ERR = e
    if _EXT is None:
        raise RuntimeError(
            "gfx950 kernels (_k8sllm_ops) are not built/loadable; run "
            "`python -m k8s_llm_monitor_amd.ops.build` (cause: %r)" % (_EXT_ERR,))
    return _EXT


def native_available() -> bool:
    try:
        native()
        return True
    except RuntimeError:
        return False


def _gpu(t: torch.Tensor) -> bool:
    return t.is_cuda


# ---------------------------------------------------------------- norms / activations

def rms_norm(x: torch.Tensor, w: torch.Tensor, eps: float, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    if not _gpu(x):
        r = ref.rms_norm(x, w, eps)
        return out.copy_(r) if out is not None else r
    if out is None:
        out = torch.empty(x.shape, dtype=x.dtype, device=x.device)
    native().rms_norm(out, x, w, eps)
    return out


def fused_add_rms_norm(x: torch.Tensor, residual: torch.Tensor, w: torch.Tensor, eps: float,
                       out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """residual <- x + residual (bf16); returns rms_norm(residual) * w."""
    if not _gpu(x):
        y, s = ref.fused_add_rms_norm(x, residual, w, eps)
        residual.copy_(s)
        return out.copy_(y) if out is not None else y
    if out is None:
        out = torch.empty(x.shape, dtype=x.dtype, device=x.device)
    native().fused_add_rms_norm(out, x, residual, w, eps)
    return out


# ---------------------------------------------------------------- decode projections (skinny GEMM)

SKINNY_MAX_M = 64
SKINNY_GROUPED_MAX_M = 128  # grouped (expert) launches over row-major weights: gemm_skinny.hip


def pack_skinny(w: torch.Tensor) -> torch.Tensor:
    """Row-major weight [N, K] -> the fragment-packed [N/16, K/32, 64, 8] layout of gemm_skinny:
    block (n-tile j, k-step s) holds, for lane l = 16 q + r, elements W[16 j + r, 32 s + 8 q : +8]
    (the v_mfma_f32_16x16x32_bf16 B operand), 1 KiB contiguous per block."""
    N, K = w.shape
    if N % 16 or K % 32:
        raise ValueError(f"pack_skinny: [{N}, {K}] needs N % 16 == 0 and K % 32 == 0")
    return w.reshape(N // 16, 16, K // 32, 4, 8).permute(0, 2, 3, 1, 4).reshape(N // 16, K // 32, 64, 8).contiguous()


def unpack_skinny(wp: torch.Tensor) -> torch.Tensor:
    nt, ks = wp.shape[0], wp.shape[1]
    return wp.reshape(nt, ks, 4, 16, 8).permute(0, 3, 1, 2, 4).reshape(nt * 16, ks * 32)


def interleave_gate_up(w13: torch.Tensor) -> torch.Tensor:
    """[gate (F rows); up (F rows)] -> per 128-row tile [64 gate | 64 up] rows (the SWIGLU
    epilogues: gate and up of an output column land in the same workgroup)."""
    F2, K = w13.shape
    F = F2 // 2
    if F % 64:
        raise ValueError("interleave_gate_up: F must be a multiple of 64")
    return w13.reshape(2, F // 64, 64, K).permute(1, 0, 2, 3).reshape(F2, K)


def deinterleave_gate_up(w: torch.Tensor) -> torch.Tensor:
    """Inverse of interleave_gate_up: per-128-row [64 gate | 64 up] -> [gate (F rows); up (F rows)]."""
    F2, K = w.shape
    return w.reshape(F2 // 128, 2, 64, K).permute(1, 0, 2, 3).reshape(F2, K)


# test / tool overrides (module attributes, not environment switches): a forced split-K factor for
# the slab-epilogue projections (real split-K slicing on tiny test shapes), and a forced waves-per-
# workgroup count for gemm_skinny (0 = the launcher's choice)
SKINNY_SPLITS_FORCE = 0
SKINNY_WAVES_FORCE = 0


def skinny_splits(N: int, K: int, target_wgs: int = 256) -> int:
    """Split-K factor for a slab-epilogue gemm_skinny: (N/64) x S workgroups ~ one per CU, each K
    slice at least 512 deep (tools/bench_skinny.py on MI355X, decode batch 1-64: S = 4 beats 2, 6
    and 8 for Llama-3-8B o/down - more slices add slab traffic to the reduce faster than they add
    weight-streaming parallelism).  ``SKINNY_SPLITS_FORCE`` (tests, tools) overrides."""
    if SKINNY_SPLITS_FORCE:
        return max(1, SKINNY_SPLITS_FORCE)
    tiles = max(1, N // 64)
    return max(1, min(K // 512, round(target_wgs / tiles)))


def skinny_workspace(max_m: int, N: int, splits: int, device) -> torch.Tensor:
    """fp32 split-K partial slabs [splits, max_m, N]."""
    return torch.empty(splits * min(max_m, SKINNY_MAX_M) * N, dtype=torch.float32, device=device)


def skinny_kchunk(K: int, S: int) -> int:
    """The K slice of each split (mirror of skinny_kchunk in gemm_skinny.hip): rounded up to whole
    128-deep wave groups where that keeps S slices, else to whole 32-deep k-steps."""
    kc = -(-K // S)
    kc128 = -(-kc // 128) * 128
    if -(-K // kc128) == S:
        return kc128
    return -(-kc // 32) * 32


def skinny_nslabs(K: int, S: int) -> int:
    return -(-K // skinny_kchunk(K, S))


# CPU forms of the skinny ops: the same packed layouts, split-K slicing and roundings as the
# kernels, so the decode control flow (and TP over gloo) is exercised by the CPU test suite.
def skinny_wdims(wp: torch.Tensor) -> tuple:
    """(N, K) of a skinny-GEMM weight: fragment-packed [N/16, K/32, 64, 8] or row-major [N, K]
    (the single resident copy, read by gemm_skinny_rm_kernel)."""
    if wp.dim() == 4:
        return wp.shape[0] * 16, wp.shape[1] * 32
    return wp.shape[0], wp.shape[1]


def _cpu_w(wp: torch.Tensor) -> torch.Tensor:
    return (unpack_skinny(wp) if wp.dim() == 4 else wp).float()


def _cpu_deinterleave(gu: torch.Tensor) -> tuple:
    M, F2 = gu.shape
    t = gu.reshape(M, F2 // 128, 2, 64)
    return t[:, :, 0].reshape(M, F2 // 2), t[:, :, 1].reshape(M, F2 // 2)


def _rows(a: torch.Tensor, rows: Optional[int] = None) -> int:
    """Valid rows of an activation: row-major [M, K], or fragment-packed [ceil(M/16), K/32, 64, 8]
    (then ``rows`` must be given)."""
    if a.dim() == 4:
        if rows is None:
            raise ValueError("a fragment-packed activation needs its row count")
        return rows
    return a.shape[0]


def _cpu_a(a: torch.Tensor, rows: Optional[int]) -> torch.Tensor:
    return unpack_skinny(a)[: _rows(a, rows)] if a.dim() == 4 else a


def pack_activation(x: torch.Tensor, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Row-major [M, K] (M <= 64) -> fragment-packed [ceil(M/16), K/32, 64, 8] (rows padded with
    zeros), the A-operand layout gemm_skinny reads with whole-line loads."""
    M, K = x.shape
    mt = -(-M // 16)
    if M % 16:
        x = torch.cat([x, x.new_zeros(mt * 16 - M, K)])
    p = pack_skinny(x)
    return out.copy_(p) if out is not None else p


def _rn_scale(rownorm, M: int, K: int) -> Optional[torch.Tensor]:
    """CPU form of the deferred RMSNorm row scale: 1 / rms per row from partial sums of squares."""
    if rownorm is None:
        return None
    ss, eps = rownorm
    return torch.rsqrt(ss[:M].float().sum(1, keepdim=True) / K + eps)


def skinny_waves() -> int:
    """Waves per gemm_skinny workgroup: 0 = the launcher's choice (8 for split-K slabs, 4 for the
    single-slice epilogues); ``SKINNY_WAVES_FORCE`` = 4 or 8 forces one (tools)."""
    return SKINNY_WAVES_FORCE


def _rn_args(rownorm) -> tuple:
    return ((None, 0.0) if rownorm is None else (rownorm[0], float(rownorm[1]))) + (skinny_waves(),)


def skinny_auto_splits(M: int, N: int, K: int) -> int:
    """Mirror of k8sllm_gemm_skinny_auto_splits: the largest power-of-two split that keeps the grid
    (64 columns per workgroup) within one workgroup per CU, K slices >= 512 deep and whole 256-deep
    rounds of the waves."""
    tiles = max(1, N // 64)
    sp = 1
    while sp < 16 and tiles * sp * 2 <= 256 and K // (sp * 2) >= 512 and K % (sp * 2 * 256) == 0:
        sp *= 2
    return sp


def skinny_linear(a: torch.Tensor, wp: torch.Tensor, out: Optional[torch.Tensor] = None,
                  nt_tiles: int = 4, rows: Optional[int] = None, rownorm: Optional[tuple] = None) -> torch.Tensor:
    """``a @ W^T`` for <= 64 rows over the fragment-packed weight, one K slice.  ``rownorm =
    (ss_part, eps)``: ``a`` holds x * norm_w (add_norm_partial) and the rows' 1/rms is applied to
    the outputs (the deferred RMSNorm)."""
    M = _rows(a, rows)
    if not _gpu(a):
        x = _cpu_a(a, rows)
        y = x.float() @ _cpu_w(wp).t()
        sc = _rn_scale(rownorm, M, x.shape[1])
        y = (y * sc if sc is not None else y).to(x.dtype)
        return out.copy_(y) if out is not None else y
    N = skinny_wdims(wp)[0]
    if out is None:
        out = torch.empty(M, N, dtype=a.dtype, device=a.device)
    native().gemm_skinny(a, wp, None, out, 1, 1, nt_tiles, M, *_rn_args(rownorm))
    return out


def skinny_swiglu(a: torch.Tensor, wp13: torch.Tensor, out: Optional[torch.Tensor] = None,
                  rows: Optional[int] = None, packed_out: bool = False,
                  rownorm: Optional[tuple] = None) -> torch.Tensor:
    """``silu(a @ Wg^T) * (a @ Wu^T)`` over a packed, gate/up-interleaved w13: [M, F], or with
    ``packed_out`` the fragment-packed [ceil(M/16), F/32, 64, 8] (the down projection's A)."""
    M = _rows(a, rows)
    F = skinny_wdims(wp13)[0] // 2
    if not _gpu(a):
        x = _cpu_a(a, rows)
        gu = x.float() @ _cpu_w(wp13).t()
        sc = _rn_scale(rownorm, M, x.shape[1])
        if sc is not None:
            gu = gu * sc
        g, u = _cpu_deinterleave(gu.to(x.dtype).float())
        y = (torch.nn.functional.silu(g) * u).to(x.dtype)
        if packed_out:
            y = pack_activation(y)
        return out.copy_(y) if out is not None else y
    if out is None:
        shape = (-(-M // 16), F // 32, 64, 8) if packed_out else (M, F)
        out = torch.empty(shape, dtype=a.dtype, device=a.device)
    native().gemm_skinny(a, wp13, None, out, 1, 3 if packed_out else 2, 4, M, *_rn_args(rownorm))
    return out


def skinny_slabs(a: torch.Tensor, wp: torch.Tensor, workspace: torch.Tensor, splits: int,
                 nt_tiles: int = 4, rows: Optional[int] = None, rownorm: Optional[tuple] = None) -> int:
    """Split-K ``a @ W^T`` into fp32 slabs [S', M, N] in ``workspace``; returns S'."""
    M = _rows(a, rows)
    if not _gpu(a):
        x = _cpu_a(a, rows)
        N, K = skinny_wdims(wp)
        if splits <= 0:
            splits = skinny_auto_splits(M, N, K)
        kc, ns = skinny_kchunk(K, splits), skinny_nslabs(K, splits)
        w = _cpu_w(wp)
        sc = _rn_scale(rownorm, M, K)
        slabs = workspace[: ns * M * N].view(ns, M, N)
        for s in range(ns):
            y = x[:, s * kc:(s + 1) * kc].float() @ w[:, s * kc:(s + 1) * kc].t()
            slabs[s] = y * sc if sc is not None else y
        return ns
    return native().gemm_skinny(a, wp, workspace, None, splits, 0, nt_tiles, M, *_rn_args(rownorm))


def skinny_grouped_swiglu(a: torch.Tensor, wp13: torch.Tensor, rows: int, out: Optional[torch.Tensor] = None
                          ) -> torch.Tensor:
    """MoE gate/up for every local expert in ONE launch (grid.z = experts): ``a`` is the shared
    fragment-packed activation [MT, K/32, 64, 8], ``wp13`` the stacked packed, gate/up-interleaved
    expert weights [E, 2F/16, K/32, 64, 8]; returns the per-expert packed SwiGLU activations
    [E, MT, F/32, 64, 8] (the grouped down projection's A)."""
    E, F = wp13.shape[0], skinny_wdims(wp13[0])[0] // 2
    mt = -(-rows // 16)
    if not _gpu(a):
        y = torch.stack([skinny_swiglu(a, wp13[e], rows=rows, packed_out=True) for e in range(E)])
        return out.copy_(y) if out is not None else y
    if out is None:
        out = torch.empty(E, mt, F // 32, 64, 8, dtype=a.dtype, device=a.device)
    native().gemm_skinny_grouped(a, wp13, None, out, 1, 3, rows, None, skinny_waves())
    return out


def skinny_grouped_slabs(act: torch.Tensor, wp2: torch.Tensor, workspace: torch.Tensor, rows: int,
                         row_w: torch.Tensor, splits: int = 1) -> int:
    """MoE down projection of every local expert in ONE launch: fp32 slabs [E * S', M, N] where
    expert e's rows are scaled by its routing weights ``row_w[:, e]`` (0 where not selected), so
    summing all slabs (add_norm_partial / reduce_slabs) IS the weighted expert combine.  Returns
    the slab count E * S'."""
    E, (N, K) = wp2.shape[0], skinny_wdims(wp2[0])
    M = rows
    if not _gpu(act):
        kc, ns = skinny_kchunk(K, splits), skinny_nslabs(K, splits)
        slabs = workspace[: E * ns * M * N].view(E * ns, M, N)
        for e in range(E):
            x = unpack_skinny(act[e])[:M].float()
            w = _cpu_w(wp2[e])
            for s in range(ns):
                slabs[e * ns + s] = (x[:, s * kc:(s + 1) * kc] @ w[:, s * kc:(s + 1) * kc].t()) * row_w[:M, e:e + 1]
        return E * ns
    return native().gemm_skinny_grouped(act, wp2, workspace, None, splits, 0, rows, row_w.contiguous(),
                                        skinny_waves())


# ---------------------------------------------------------------- decode GEMM, shared-A design (gemm_decode.hip)

def interleave_gate_up8(w13: torch.Tensor) -> torch.Tensor:
    """[gate (F rows); up (F rows)] -> per 16-row n-tile [8 gate | 8 up] rows: the DEC_SWIGLU8
    epilogue finds a feature's gate and up in lanes l and l ^ 8 of one accumulator."""
    F2, K = w13.shape
    F = F2 // 2
    if F % 8:
        raise ValueError("interleave_gate_up8: F must be a multiple of 8")
    return w13.reshape(2, F // 8, 8, K).permute(1, 0, 2, 3).reshape(F2, K)


def deinterleave_gate_up8(w: torch.Tensor) -> torch.Tensor:
    F2, K = w.shape
    return w.reshape(F2 // 16, 2, 8, K).permute(1, 0, 2, 3).reshape(F2, K)


# (splits, n-tiles per wave, waves, weight ring depth) per decode projection shape (N, K) at
# M <= 64: ~256 equal workgroups (measured: tools/bench_decode_gemm.py,
# profiles/r04/decode_gemm_sweep.jsonl).  Shapes not listed get an automatic pick.
DEC_TABLE: dict = {
    # Llama-3-8B at TP=1 (profiles/r04/decode_gemm_sweep_v1.jsonl, M = 64 / M = 1 us):
    # qkv: 6 waves -> 64 column groups x 4 splits = 256 workgroups (8 waves left 64 CUs idle):
    # 12.1 vs 13.8 us at M = 64, 9.8 vs 11.0 at M = 1 (decode_gemm_qkv_6waves.jsonl)
    (6144, 4096, 0): (4, 1, 6, 8),      # qkv      12.1 / 9.8    (row-major skinny 13.5 / 10.6)
    (4096, 4096, 0): (8, 1, 8, 8),      # o         9.6 / 7.5    (10.2 / 7.5)
    (28672, 4096, 2): (1, 1, 7, 8),     # gate_up  39.9 / 38.1   (47.9 / 40.0)
    (4096, 14336, 0): (8, 1, 8, 8),     # down     22.3 / 19.0   (24.3 / 19.9)
    (128256, 4096, 1): (1, 4, 8, 4),    # LM head 173.8 / 166.0  (hipBLASLt 202.2 / 176.2)
}



def dec_config(N: int, K: int, epi: int, experts: int = 1) -> Optional[tuple]:
    """Launch configuration of gemm_dec for a weight [N, K]: (splits, ntw, waves, depth) or None
    when no configuration tiles the shape (the caller keeps gemm_skinny).  The candidates are the
    (ntw, waves, depth) forms gemm_decode.hip instantiates: every Llama-3-8B / 70B / Mixtral
    projection and LM head at TP 1..8 picks one of them (tools/bench_decode_gemm.py passes ``cfg``
    to dec_gemm to time others).  ``experts`` > 1: a grouped launch (grid.z = expert), whose
    workgroup count is per expert times experts (Mixtral down: 32 column groups x 8 experts, no
    split - the expert slabs are the split)."""
    hit = DEC_TABLE.get((N, K, epi)) if experts == 1 else None
    if hit is not None:
        return hit
    ntiles, ksteps = N // 16, K // 32
    cands = ([(1, 1, 7, 8), (1, 1, 7, 16), (1, 1, 8, 16)] if epi == 2 else
             [(1, 4, 8, 4), (1, 3, 8, 8), (1, 2, 8, 8), (1, 1, 8, 8)] if epi == 1 else
             [(s, ntw, w, d) for s in (1, 2, 4, 8, 16) for (ntw, w, d) in ((1, 8, 8), (1, 4, 16), (1, 4, 8))])
    best = None
    for s, ntw, w, d in cands:
        if experts > 1 and s > 1:  # grouped: the per-expert slabs are the split (workspace E x M x N)
            continue
        it = max(d, 8)
        if (epi == 0 and ntiles % (ntw * w)) or K % s or (ksteps // s) % it or ksteps % s:
            continue
        wgs = -(-ntiles // (ntw * w)) * s * experts
        # ~256 workgroups; for split-K slabs 8-wave workgroups of one n-tile per wave were the
        # fastest within 64 workgroups of that (the sweep), then fewer K splits (slab traffic)
        far = abs(wgs - 256) if wgs <= 512 else 10_000 + wgs
        key = ((far > 64, -w, far, s) if epi == 0 else (far, s))
        if best is None or key < best[0]:
            best = (key, (s, ntw, w, d))
    return best[1] if best else None


def dec_available(N: int, K: int, epi: int) -> bool:
    return dec_config(N, K, epi) is not None


def dec_gemm(a: torch.Tensor, wp: torch.Tensor, epi: int, rows: int, workspace: Optional[torch.Tensor] = None,
             out: Optional[torch.Tensor] = None, rownorm: Optional[tuple] = None,
             cfg: Optional[tuple] = None) -> int:
    """gemm_dec over a fragment-packed activation ``a`` and packed weight ``wp`` (decode-only copy).
    epi 0: fp32 split-K slabs into ``workspace`` [S, M, N], returns S; epi 1: ``out`` [M, N] bf16;
    epi 2: ``out`` packed SwiGLU [ceil(M/16), F/32, 64, 8] over an interleave_gate_up8 weight.
    ``rownorm = (ss_part, eps)``: deferred RMSNorm of the A rows (add_norm_partial).  CPU: the fp32
    reference with the same split-K slicing."""
    N, K = skinny_wdims(wp)
    M = rows
    if cfg is None:
        cfg = dec_config(N, K, epi)
    if cfg is None:
        raise ValueError(f"gemm_dec: no configuration for N={N} K={K} epi={epi}")
    S, ntw, waves, depth = cfg
    if not _gpu(a):
        x = _cpu_a(a, rows).float()
        w = _cpu_w(wp)
        sc = _rn_scale(rownorm, M, K)
        if epi == 0:
            kc = K // S
            slabs = workspace[: S * M * N].view(S, M, N)
            for s in range(S):
                y = x[:, s * kc:(s + 1) * kc] @ w[:, s * kc:(s + 1) * kc].t()
                slabs[s] = y * sc if sc is not None else y
            return S
        y = x @ w.t()
        if sc is not None:
            y = y * sc
        if epi == 1:
            out[:M].copy_(y.to(out.dtype))
            return 1
        gu = deinterleave_gate_up8(y.to(a.dtype).float().t()).t()
        g, u = gu[:, : N // 2], gu[:, N // 2:]
        out.copy_(pack_activation((torch.nn.functional.silu(g) * u).to(a.dtype)))
        return 1
    rn = (None, 0.0) if rownorm is None else (rownorm[0], float(rownorm[1]))
    r = native().gemm_dec(a, wp, workspace, out, S, epi, ntw, waves, depth, M, *rn)
    if r < 0:
        raise RuntimeError(f"gemm_dec: configuration {cfg} not compiled for N={N} K={K} epi={epi}")
    return r


def dec_gemm_grouped(a: torch.Tensor, wp: torch.Tensor, epi: int, rows: int, workspace: Optional[torch.Tensor] = None,
                     out: Optional[torch.Tensor] = None, row_w: Optional[torch.Tensor] = None,
                     cfg: Optional[tuple] = None) -> int:
    """gemm_dec over every local expert of a MoE layer in ONE launch (grid.z = expert): ``wp``
    [E, N/16, K/32, 64, 8] (packed per expert, gate/up interleave_gate_up8 for epi 2); ``a`` packed
    [ceil(M/16), K/32, 64, 8] shared by the experts (gate_up) or [E, ...] per expert (down).
    epi 2: ``out`` [E, ceil(M/16), F/32, 64, 8] packed SwiGLU; epi 0: fp32 slabs [E * S, M, N] in
    ``workspace`` scaled by ``row_w`` [M, E] (routing weights, 0 where a row skipped the expert),
    returns E * S - the residual-add kernel's slab sum is the expert combine."""
    E = wp.shape[0]
    N, K = wp.shape[1] * 16, wp.shape[2] * 32
    M = rows
    if cfg is None:
        cfg = dec_config(N, K, epi, experts=E)
    if cfg is None:
        raise ValueError(f"gemm_dec_grouped: no configuration for N={N} K={K} epi={epi}")
    S, ntw, waves, depth = cfg
    if not _gpu(a):
        for e in range(E):
            ae = a[e] if a.dim() == 5 else a
            if epi == 2:
                dec_gemm(ae, wp[e], 2, M, out=out[e], cfg=cfg)
            else:
                ws = workspace[e * S * M * N: (e + 1) * S * M * N]
                dec_gemm(ae, wp[e], 0, M, workspace=ws, cfg=cfg)
                if row_w is not None:
                    ws.view(S, M, N).mul_(row_w[:M, e].float().view(1, M, 1))
        return E * S if epi == 0 else 1
    r = native().gemm_dec_grouped(a, wp, workspace, out, S, epi, ntw, waves, depth, M, row_w)
    if r < 0:
        raise RuntimeError(f"gemm_dec_grouped: configuration {cfg} not compiled for N={N} K={K} epi={epi}")
    return r


def dec_gemm_rc(a: torch.Tensor, wp: torch.Tensor, rows: int, residual: torch.Tensor, norm_w: torch.Tensor,
                eps: float) -> Optional[tuple]:
    """Row-complete decode GEMM (gemm_dec_rc_kernel) for a residual-producing projection:
    ``residual += a . W^T`` in place (no split-K slabs) and the next GEMM's deferred-RMSNorm
    operands in the same launch: returns ``(xw, (ss, eps))`` - xw = residual * norm_w
    fragment-packed, ss [rows, N/16] per-16-column sums of squares - or None where the kernel does
    not tile the shape (the caller keeps slabs + add_norm_partial).  CPU: the fp32 reference with
    the same 8 K-slices summed in slice order."""
    N, K = skinny_wdims(wp)
    M = rows
    if K % 256 or N % 32 or M > 64:
        return None
    xw = packed_empty(M, N, residual.dtype, residual.device)
    ss = torch.empty(M, N // 16, dtype=torch.float32, device=residual.device)
    if not _gpu(a):
        x = _cpu_a(a, rows).float()
        w = _cpu_w(wp)
        kc = K // 8
        h = residual[:M].float()
        for s in range(8):
            h = h + x[:, s * kc:(s + 1) * kc] @ w[:, s * kc:(s + 1) * kc].t()
        residual[:M] = h.to(residual.dtype)
        v = residual[:M].float()
        ss.copy_((v * v).view(M, N // 16, 16).sum(-1))
        xw.copy_(pack_activation((v * norm_w.float()).to(residual.dtype)))
        return xw, (ss, eps)
    if not native().gemm_dec_rc(a, wp, residual, norm_w, xw, ss, rows):
        return None
    return xw, (ss, eps)


def add_norm_partial(residual: torch.Tensor, workspace: Optional[torch.Tensor], nslabs: int, norm_w: torch.Tensor,
                     out: Optional[torch.Tensor] = None, ss_part: Optional[torch.Tensor] = None,
                     packed: bool = True) -> tuple:
    """Residual update with a deferred RMSNorm: ``residual <- residual + sum of slabs``;
    returns ``(residual * norm_w`` (fragment-packed by default), ``ss_part [M, d/512])`` for a
    consumer skinny GEMM called with ``rownorm=(ss_part, eps)``.  One wave per 512 columns: the
    norm's row reduction is left to the consumer's epilogue."""
    M, d = residual.shape
    if ss_part is None:
        ss_part = torch.empty(M, d // 512, dtype=torch.float32, device=residual.device)
    if out is None:
        out = packed_empty(M, d, residual.dtype, residual.device) if packed else torch.empty_like(residual)
    if not _gpu(residual):
        if nslabs:
            s = workspace[: nslabs * M * d].view(nslabs, M, d).sum(0)
            residual.copy_((residual.float() + s).to(residual.dtype))
        v = residual.float()
        ss_part.copy_((v * v).view(M, d // 512, 512).sum(-1))
        y = (v * norm_w.float()).to(residual.dtype)
        out.copy_(pack_activation(y) if out.dim() == 4 else y)
        return out, ss_part
    native().add_norm_partial(out, residual, workspace, nslabs, norm_w, ss_part)
    return out, ss_part


def reduce_slabs(workspace: torch.Tensor, nslabs: int, M: int, N: int, dtype=torch.bfloat16,
                 out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Sum of ``nslabs`` split-K slabs [nslabs, M, N] -> [M, N] in ``dtype`` (TP>1 tails, before
    the all-reduce)."""
    if not _gpu(workspace):
        y = workspace[: nslabs * M * N].view(nslabs, M, N).sum(0).to(dtype)
        return out.copy_(y) if out is not None else y
    if out is None:
        out = torch.empty(M, N, dtype=dtype, device=workspace.device)
    native().reduce_slabs(out, workspace, nslabs)
    return out


def reduce_add_rms_norm(out: torch.Tensor, residual: torch.Tensor, workspace: Optional[torch.Tensor], nslabs: int,
                        norm_w: torch.Tensor, eps: float, packed_out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """``residual <- residual + sum of slabs`` (rounded to the residual dtype), ``out <- rms_norm``.
    ``nslabs = 0``: a plain RMSNorm of ``residual``.  A 4-D ``out`` is written fragment-packed
    ([ceil(M/16), d/32, 64, 8], the next skinny GEMM's A operand); ``packed_out``: a second,
    packed copy of the same rows (same launch)."""
    if not _gpu(residual):
        M, N = residual.shape
        if nslabs:
            s = workspace[: nslabs * M * N].view(nslabs, M, N).sum(0)
            residual.copy_((residual.float() + s).to(residual.dtype))
        y = ref.rms_norm(residual, norm_w, eps)
        if packed_out is not None:
            packed_out.copy_(pack_activation(y))
        return out.copy_(pack_activation(y) if out.dim() == 4 else y)
    native().reduce_add_rms_norm(out, residual, workspace, nslabs, norm_w, eps, packed_out)
    return out


def packed_empty(M: int, K: int, dtype, device) -> torch.Tensor:
    """Uninitialised fragment-packed activation buffer [ceil(M/16), K/32, 64, 8]."""
    return torch.empty(-(-M // 16), K // 32, 64, 8, dtype=dtype, device=device)


def proj_add_rms_norm(a: torch.Tensor, wp: torch.Tensor, residual: torch.Tensor, norm_w: torch.Tensor, eps: float,
                      workspace: Optional[torch.Tensor] = None, splits: Optional[int] = None,
                      out: Optional[torch.Tensor] = None, rows: Optional[int] = None,
                      packed_out: bool = False) -> torch.Tensor:
    """The decode tail of an attention or MLP block in one GEMM + one reduce:
    ``residual <- residual + a @ W^T``; returns ``rms_norm(residual) * norm_w`` (row-major, or
    fragment-packed with ``packed_out``).  GPU: gemm_skinny (packed ``wp``, split-K fp32 slabs)
    then reduce_add_rms_norm."""
    M, (N, K) = _rows(a, rows), skinny_wdims(wp)
    if splits is None:
        splits = 0  # automatic (launcher)
    if workspace is None:
        workspace = skinny_workspace(M, N, splits or skinny_auto_splits(M, N, K), a.device)
    s = skinny_slabs(a, wp, workspace, splits, rows=M)
    if out is None:
        out = (packed_empty(M, N, residual.dtype, a.device) if packed_out
               else torch.empty(M, N, dtype=residual.dtype, device=a.device))
    return reduce_add_rms_norm(out, residual, workspace, s, norm_w, eps)


def gemm_skinny(a: torch.Tensor, w: torch.Tensor, splits: int = 1) -> torch.Tensor:
    """``a @ w^T`` through the skinny kernel from a row-major weight (tests / tools)."""
    wp = pack_skinny(w)
    if splits == 1:
        return skinny_linear(a, wp)
    M, N = a.shape[0], w.shape[0]
    ws = skinny_workspace(M, N, splits, a.device)
    s = skinny_slabs(a, wp, ws, splits)
    return reduce_slabs(ws, s, M, N, a.dtype)


def layer_norm(x, w, b, eps):
    if not _gpu(x):
        return ref.layer_norm(x, w, b, eps)
    x = x.contiguous()
    out = torch.empty_like(x)
    native().layer_norm(out, x, w, b, eps)
    return out


def silu_mul(x: torch.Tensor, out: Optional[torch.Tensor] = None, interleaved: bool = False) -> torch.Tensor:
    """silu(gate) * up over [.., 2F] gate_up activations: [F gate | F up], or ``interleaved``
    [64 gate | 64 up] per 128 columns (the output of the single resident, interleaved w13)."""
    if not _gpu(x):
        y = ref.silu_mul(x, interleaved)
        return out.copy_(y) if out is not None else y
    if out is None:
        out = torch.empty(*x.shape[:-1], x.shape[-1] // 2, dtype=x.dtype, device=x.device)
    native().silu_mul(out, x.contiguous(), interleaved)
    return out


def gelu_tanh(x: torch.Tensor) -> torch.Tensor:
    if not _gpu(x):
        return ref.gelu_tanh(x)
    x = x.contiguous()
    out = torch.empty_like(x)
    native().gelu_tanh(out, x)
    return out


def embedding(ids: torch.Tensor, weight: torch.Tensor, vocab_start: int = 0,
              out: Optional[torch.Tensor] = None) -> torch.Tensor:
    if not _gpu(weight):
        return ref.embedding(ids, weight, vocab_start)
    if out is None:
        out = torch.empty(ids.numel(), weight.shape[1], dtype=weight.dtype, device=weight.device)
    native().embedding(out, ids, weight, vocab_start)
    return out


def embed_norm_partial(ids: torch.Tensor, weight: torch.Tensor, norm_w: torch.Tensor,
                       src: Optional[torch.Tensor] = None, prev: Optional[torch.Tensor] = None,
                       packed: bool = True) -> tuple:
    """The decode step's front end: the (pipelined, see :func:`resolve_ids`) input ids' embedding
    rows and the first layer's deferred-norm operands - ``(residual [M, d], residual * norm_w
    (fragment-packed), ss_part [M, d/512])``, what embedding + add_norm_partial(nslabs=0) return,
    in one launch."""
    M, d = ids.numel(), weight.shape[1]
    if not _gpu(weight):
        if src is not None:
            ids = resolve_ids(ids, src, prev)
        res = ref.embedding(ids, weight, 0).contiguous()
        xw, ss = add_norm_partial(res, None, 0, norm_w, packed=packed)
        return res, xw, ss
    res = torch.empty(M, d, dtype=weight.dtype, device=weight.device)
    ss = torch.empty(M, d // 512, dtype=torch.float32, device=weight.device)
    out = packed_empty(M, d, weight.dtype, weight.device) if packed else torch.empty_like(res)
    native().embed_norm_partial(out, res, ids, src, prev, weight, norm_w, ss)
    return res, out, ss


def resolve_ids(ids: torch.Tensor, src: torch.Tensor, prev: torch.Tensor,
                out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Decode input ids under pipelining: ``prev[src[i]]`` where ``src[i] >= 0`` (the token the
    previous step sampled in that row, still on the device), else ``ids[i]``."""
    if not _gpu(ids):
        return torch.where(src >= 0, prev.index_select(0, src.clamp(min=0).long()), ids)
    if out is None:
        out = torch.empty_like(ids)
    native().resolve_ids(out, ids, src, prev)
    return out


# ---------------------------------------------------------------- attention

def rope_and_cache(qkv: torch.Tensor, positions: torch.Tensor, cos_sin: torch.Tensor,
                   k_cache: Optional[torch.Tensor], v_cache: Optional[torch.Tensor],
                   slot_mapping: Optional[torch.Tensor], Hq: int, Hkv: int, D: int,
                   apply_rope: bool = True, partial: Optional[torch.Tensor] = None, nslabs: int = 0) -> None:
    """In place: rotate q and k inside the fused QKV rows; write k, v into the paged cache.
    With ``partial`` (GPU), the QKV values are first reduced from ``nslabs`` fp32 split-K slabs
    [nslabs, T, (Hq+2Hkv)*D] (skinny_slabs) and the reduced rows are written to ``qkv``."""
    if not _gpu(qkv):
        if partial is not None:
            T, n = qkv.shape[0], qkv.shape[1]
            qkv.copy_(partial[: nslabs * T * n].view(nslabs, T, n).sum(0).to(qkv.dtype))
        ref.rope_and_cache(qkv, positions, cos_sin, k_cache, v_cache, slot_mapping, Hq, Hkv, D, apply_rope)
        return
    empty = _empty_i32(qkv.device)
    native().rope_and_cache(qkv, positions, cos_sin,
                            k_cache if k_cache is not None else empty,
                            v_cache if v_cache is not None else empty,
                            slot_mapping if slot_mapping is not None else empty,
                            Hq, Hkv, D, apply_rope, partial, nslabs)


_EMPTY = {}


def _empty_i32(device) -> torch.Tensor:
    t = _EMPTY.get(device)
    if t is None:
        t = _EMPTY[device] = torch.empty(0, dtype=torch.int32, device=device)
    return t


MAX_SPLITS = 64


def decode_splits(batch: int, Hkv: int, n_cu: int = 256) -> int:
    """Splits per (sequence, kv head) for paged_decode: aim for ~one workgroup per CU in total.

    Measured on MI355X (tools/bench_decode.py, ctx 1.8k-6k): batch 64 x 8 kv heads is best
    unsplit (83 us, 5.7 TB/s - a merge launch and extra partial traffic only cost), batch 8 at 4
    splits, batch 1 at 16-32 splits."""
    return max(1, min(32, round(n_cu / max(1, batch * Hkv))))


# split partials of paged_decode_fused merged inside the attention launch by the last-arriving
# split (no paged_decode_reduce launch); the decode workspace carries the hand-off counters
DECODE_MERGE = True


def decode_workspace(max_batch: int, Hq: int, D: int, max_model_len: int = 0, device=None, Hkv: Optional[int] = None):
    """fp32 partials of the split-K decode kernel: [B, Hq, MAX_SPLITS, D] and [.., 2], plus the
    in-launch merge's (sequence, kv head) counters (int32, zero; each launch leaves them zero)."""
    part_out = torch.empty(max_batch, Hq, MAX_SPLITS, D, dtype=torch.float32, device=device)
    part_ml = torch.empty(max_batch, Hq, MAX_SPLITS, 2, dtype=torch.float32, device=device)
    ctr = torch.zeros(max_batch * Hq, dtype=torch.int32, device=device)
    return part_out, part_ml, ctr


def paged_decode(q: torch.Tensor, k_cache: torch.Tensor, v_cache: torch.Tensor, block_tables: torch.Tensor,
                 seq_lens: torch.Tensor, Hq: int, Hkv: int, D: int, scale: float,
                 workspace: Optional[tuple] = None, out: Optional[torch.Tensor] = None,
                 splits: Optional[int] = None) -> torch.Tensor:
    if not _gpu(q):
        r = cpu_attn.paged_decode(q, k_cache, v_cache, block_tables, seq_lens, Hq, Hkv, D, scale)
        if out is not None and out.dim() == 4:  # fragment-packed output (gemm_skinny A operand)
            r = pack_activation(r)
        return out.copy_(r) if out is not None else r
    B = seq_lens.shape[0]
    if workspace is None:
        workspace = decode_workspace(B, Hq, D, device=q.device)
    if out is None:
        out = torch.empty(B, Hq * D, dtype=q.dtype, device=q.device)
    S = splits or decode_splits(B, Hkv)
    native().paged_decode(out, q, k_cache, v_cache, block_tables, seq_lens, workspace[0], workspace[1],
                          Hq, Hkv, D, scale, S)
    return out


def paged_decode_fused(slabs: torch.Tensor, nslabs: int, positions: torch.Tensor, cos_sin: torch.Tensor,
                       slot_mapping: Optional[torch.Tensor], k_cache: torch.Tensor, v_cache: torch.Tensor,
                       block_tables: torch.Tensor, seq_lens: torch.Tensor, Hq: int, Hkv: int, D: int, scale: float,
                       workspace: Optional[tuple] = None, out: Optional[torch.Tensor] = None,
                       splits: Optional[int] = None) -> torch.Tensor:
    """paged_decode with rope_and_cache folded in: the new token's q / k / v are the sum of the qkv
    projection's ``nslabs`` fp32 split-K slabs [nslabs, B, (Hq + 2 Hkv) * D] (skinny_slabs),
    rounded to the cache dtype, q / k rotated at ``positions``, k / v written to the cache at
    ``slot_mapping``; attention over the cached tokens plus the new one (D = 128 on the GPU)."""
    B = seq_lens.shape[0]
    if not _gpu(slabs):
        n = (Hq + 2 * Hkv) * D
        qkv = slabs[: nslabs * B * n].view(nslabs, B, n).sum(0).to(k_cache.dtype)
        ref.rope_and_cache(qkv, positions, cos_sin, k_cache, v_cache, slot_mapping, Hq, Hkv, D, True)
        return paged_decode(qkv, k_cache, v_cache, block_tables, seq_lens, Hq, Hkv, D, scale, out=out)
    if workspace is None:
        workspace = decode_workspace(B, Hq, D, device=slabs.device)
    if out is None:
        out = torch.empty(B, Hq * D, dtype=k_cache.dtype, device=slabs.device)
    S = splits or decode_splits(B, Hkv)
    merge = workspace[2] if DECODE_MERGE and len(workspace) > 2 else _empty_i32(slabs.device)
    native().paged_decode_fused(out, slabs, nslabs, positions, cos_sin,
                                slot_mapping if slot_mapping is not None else _empty_i32(slabs.device),
                                k_cache, v_cache, block_tables, seq_lens, workspace[0], workspace[1], Hq, Hkv, D,
                                scale, S, merge)
    return out


def prefill_qblocks(cu_seqlens_cpu: list[int], block: int = 128, ctx_starts: Optional[list[int]] = None,
                    order: str = "seq") -> tuple[list[int], list[int]]:
    """Q-block schedule for flash_prefill: (seq index, first q row) per 128-row block.  A block's
    work is its causal key span: the sequence's cached prefix (``ctx_starts``, chunked prefill)
    plus its first row.

    ``order="seq"`` (the engine's, sequence-major): the longest sequence first, each sequence's
    blocks heaviest first.  The workgroups resident on one XCD at a time (one kv head's) then cover
    one or two sequences, whose K/V stay in that XCD's 4 MiB L2, and the grid still ends on light
    blocks: 10 x 1609 tokens 276.7 vs 295.1 us, 64 x 1609 1788 vs 1934 us
    (profiles/r04/flash_qb_order_nw.jsonl).  ``work``: all blocks heaviest first across sequences,
    so the residents span ~10 sequences' K/V."""
    items = []
    for i in range(len(cu_seqlens_cpu) - 1):
        n = cu_seqlens_cpu[i + 1] - cu_seqlens_cpu[i]
        c = ctx_starts[i] if ctx_starts is not None else 0
        for s in range(0, n, block):
            items.append((c + s, s, i, c + n))
    if order == "seq":
        items.sort(key=lambda t: (-t[3], t[2], -t[0]))
    else:
        items.sort(key=lambda t: -t[0])
    return [t[2] for t in items], [t[1] for t in items]


def flash_prefill(qkv: torch.Tensor, cu_seqlens: torch.Tensor, Hq: int, Hkv: int, D: int, scale: float,
                  qblocks: Optional[tuple[torch.Tensor, torch.Tensor]] = None,
                  out: Optional[torch.Tensor] = None, paged: Optional[tuple] = None) -> torch.Tensor:
    """Causal varlen attention of the prefill rows.  ``paged = (ctx_start, k_cache, v_cache,
    block_tables)``: each sequence's rows are its NEW tokens at positions ctx_start.. and the
    keys/values (cached prefix + new) are read from the paged cache."""
    if not _gpu(qkv):
        if paged is not None:
            cs, kc, vc, bt = paged
            return cpu_attn.paged_prefill(qkv, cu_seqlens, cs, kc, vc, bt, Hq, Hkv, D, scale)
        return cpu_attn.flash_prefill(qkv, cu_seqlens, Hq, Hkv, D, scale)
    if qblocks is None:
        qs, st = prefill_qblocks(cu_seqlens.tolist())
        qblocks = (torch.tensor(qs, dtype=torch.int32, device=qkv.device),
                   torch.tensor(st, dtype=torch.int32, device=qkv.device))
    if out is None:
        out = torch.empty(qkv.shape[0], Hq * D, dtype=qkv.dtype, device=qkv.device)
    if paged is not None:
        cs, kc, vc, bt = paged
        native().flash_prefill(out, qkv, cu_seqlens, qblocks[0], qblocks[1], Hq, Hkv, D, scale, cs, kc, vc, bt)
    else:
        native().flash_prefill(out, qkv, cu_seqlens, qblocks[0], qblocks[1], Hq, Hkv, D, scale, None, None, None,
                               None)
    return out


# ---------------------------------------------------------------- sampling

def sample(logits: torch.Tensor, temperature: Optional[torch.Tensor] = None, top_k: Optional[torch.Tensor] = None,
           top_p: Optional[torch.Tensor] = None, rng: Optional[torch.Tensor] = None,
           out: Optional[torch.Tensor] = None, advance: bool = False) -> torch.Tensor:
    """Next tokens [B] int32.  temperature <= 0 (or None) is greedy.  ``advance``: bump the RNG
    counter ``rng[1]`` after drawing (on the GPU inside the final sampling kernel - no extra
    launch inside a captured decode step)."""
    if not _gpu(logits):
        r = _sample_cpu(logits, temperature, top_k, top_p, rng)
        if advance and rng is not None:
            rng[1] += 1
        return out.copy_(r) if out is not None else r
    if out is None:
        out = torch.empty(logits.shape[0], dtype=torch.int32, device=logits.device)
    native().sample(out, logits, temperature, top_k, top_p, rng, advance and rng is not None)
    return out


def _sample_cpu(logits, temperature, top_k, top_p, rng):
    B = logits.shape[0]
    res = torch.empty(B, dtype=torch.int32)
    gen = torch.Generator().manual_seed(int(rng[0]) * 1000003 + int(rng[1])) if rng is not None else None
    for b in range(B):
        t = float(temperature[b]) if temperature is not None else 0.0
        x = logits[b].float()
        if t <= 0:
            res[b] = int(x.argmax())
            continue
        x = x / t
        if top_k is not None and 0 < int(top_k[b]) < x.numel():
            kth = torch.topk(x, int(top_k[b])).values[-1]
            x = x.masked_fill(x < kth, float("-inf"))
        if top_p is not None and float(top_p[b]) < 1.0:
            p = torch.softmax(x, -1)
            sp, si = torch.sort(p, descending=True)
            keep = torch.cumsum(sp, 0) - sp < float(top_p[b])
            mask = torch.zeros_like(p, dtype=torch.bool)
            mask[si[keep]] = True
            x = x.masked_fill(~mask, float("-inf"))
        res[b] = int(torch.multinomial(torch.softmax(x, -1), 1, generator=gen))
    return res


# ---------------------------------------------------------------- mixture of experts

def moe_route(router_logits: torch.Tensor, k: int, renorm: bool = True):
    if not _gpu(router_logits):
        return ref.moe_route(router_logits, k, renorm)
    T = router_logits.shape[0]
    lf = router_logits.float().contiguous()
    ids = torch.empty(T, k, dtype=torch.int32, device=lf.device)
    w = torch.empty(T, k, dtype=torch.float32, device=lf.device)
    native().moe_route(lf, ids, w, renorm)
    return ids, w


def moe_router(x: torch.Tensor, router_w: torch.Tensor, k: int, renorm: bool = True) -> tuple:
    """MoE decode routing in one launch: ``(ids [T, k] int32, w [T, k] fp32, wd [T, E] fp32)`` -
    the top-k experts of bf16(x . router_w^T), their (renormalised) softmax weights, and the dense
    per-expert weight rows (0 where an expert was not chosen) for the grouped expert kernels."""
    T, E = x.shape[0], router_w.shape[0]
    if not _gpu(x) or E > 16:
        ids, w = moe_route(torch.nn.functional.linear(x, router_w).float(), k, renorm)
        wd = torch.zeros(T, E, dtype=torch.float32, device=x.device).scatter_(1, ids.long(), w)
        return ids, w, wd
    ids = torch.empty(T, k, dtype=torch.int32, device=x.device)
    w = torch.empty(T, k, dtype=torch.float32, device=x.device)
    wd = torch.empty(T, E, dtype=torch.float32, device=x.device)
    native().moe_router(x.contiguous(), router_w, ids, w, wd, renorm)
    return ids, w, wd


def moe_align(ids: torch.Tensor, E: int):
    if not _gpu(ids) or E > 16:
        return ref.moe_align(ids, E)
    n = ids.numel()
    offsets = torch.empty(E + 1, dtype=torch.int32, device=ids.device)
    sorted_idx = torch.empty(n, dtype=torch.int32, device=ids.device)
    inv_idx = torch.empty(n, dtype=torch.int32, device=ids.device)
    native().moe_align(ids.contiguous(), E, offsets, sorted_idx, inv_idx)
    return offsets, sorted_idx, inv_idx


def gather_rows(x: torch.Tensor, idx: torch.Tensor, div: int = 1) -> torch.Tensor:
    if not _gpu(x):
        return x[(idx.long() // div)]
    out = torch.empty(idx.numel(), x.shape[1], dtype=x.dtype, device=x.device)
    native().gather_rows(out, x.contiguous(), idx, div)
    return out


def moe_grouped_gemm(x: torch.Tensor, w: torch.Tensor, offsets: torch.Tensor, swiglu: bool = False,
                     out: Optional[torch.Tensor] = None, zero_fill: bool = True) -> torch.Tensor:
    """All experts' GEMMs in one launch over expert-sorted rows: ``x`` [rows, K], ``w`` [E, N, K],
    ``offsets`` [E + 1] int32 absolute row offsets of the experts' rows in ``x`` (moe_align, may be
    a slice for this rank's experts).  ``swiglu``: ``w`` is gate/up-interleaved and the result is
    silu(gate) * up [rows, N / 2].  Rows of other experts are left as in ``out`` (zeros when
    allocated here).  GPU: no host synchronisation (gemm_tile.hip 256 x 256 tiles where N % 256 == 0,
    else moe_gemm.hip).  A fragment-packed ``w`` [E, N/16, K/32, 64, 8] (ONE_LAYOUT; ``swiglu=8``:
    the per-16 gate/up pairing) always takes the tile kernel."""
    if w.dim() == 5:
        if out is None:
            alloc = torch.zeros if zero_fill else torch.empty
            out = alloc(x.shape[0], w.shape[1] * 8 if swiglu else w.shape[1] * 16, dtype=x.dtype, device=x.device)
        return gemm_tile(x, w, offsets, swiglu=swiglu, out=out, algo=TILE_ALGO)
    E, N, K = w.shape
    if out is None:  # zero_fill=False when ``offsets`` covers every row (all experts are local)
        alloc = torch.zeros if zero_fill else torch.empty
        out = alloc(x.shape[0], N // 2 if swiglu else N, dtype=x.dtype, device=x.device)
    if not _gpu(x):
        off = offsets.tolist()
        for e in range(E):
            a, b = off[e], off[e + 1]
            if b > a:
                y = torch.nn.functional.linear(x[a:b].float(), w[e].float()).to(x.dtype)
                out[a:b] = silu_mul(y, interleaved=True) if swiglu else y
        return out
    if N % 256 == 0 and K % 64 == 0 and N * K * 2 < (1 << 31):
        # the 256 x 256 tile kernel (gemm_tile.hip): 1.12-1.15 PF/s on Mixtral's expert shapes
        # against 0.86-0.94 for the 128-tile kernel below (profiles/r02/gemm_tile_vs_hipblaslt.jsonl)
        native().gemm_tile(out, x.contiguous(), w, offsets.contiguous(), swiglu, TILE_ALGO)
    else:
        native().moe_grouped_gemm(out, x.contiguous(), w, offsets.contiguous(), swiglu)
    return out


def gemm_tile(x: torch.Tensor, w: torch.Tensor, offsets: Optional[torch.Tensor] = None, swiglu: bool = False,
              out: Optional[torch.Tensor] = None, algo: int = 0, rope: Optional[tuple] = None,
              rowscale: Optional[tuple] = None) -> torch.Tensor:
    """Prefill-sized ``x @ w^T`` on the 256 x 256 MFMA tile kernel (csrc/gemm_tile.hip).

    Dense: ``w`` [N, K].  Grouped: ``w`` [E, N, K] and ``offsets`` [E + 1] int32 device offsets of
    each expert's rows in the expert-sorted ``x`` (moe_align; a slice for this rank's experts) - no
    host synchronisation.  ``swiglu``: ``w`` is gate/up-interleaved (interleave_gate_up) and the
    result is silu(gate) * up [M, N / 2].  Grouped rows outside the offsets are left as in ``out``
    (zeros when allocated here).  ``rope = (positions [M] int32, cos_sin [P, 128] fp32, heads)``
    (dense, N % 128 == 0): the epilogue applies rotate-half RoPE (head_dim 128) to output heads
    0 .. heads - 1 of each row at its position, on the bf16-rounded product.
    ``rowscale = (ss_part [M, K / 128] fp32, eps)`` (dense, with ``swiglu`` or ``rope``, schedule 1):
    the deferred half of an RMSNorm - every row of the product is multiplied by
    rsqrt(sum(ss_part[row]) / K + eps) before the epilogue (``x`` holds the norm's weighted input,
    gemm_tile_resid's ``hw``).
    ``w`` may also be fragment-packed (pack_skinny: [N/16, K/32, 64, 8], grouped [E, ...]): the
    decode GEMMs' layout, consumed as is (every W DMA piece one contiguous 1-KiB block).
    ``swiglu=8``: the gate/up rows are interleaved per 16 (interleave_gate_up8, the decode GEMMs'
    SwiGLU copy) instead of per 128 - prefill and decode then share one weight."""
    M = x.shape[0]
    packed = w.dim() == (5 if offsets is not None else 4)
    N = w.shape[-4] * 16 if packed else w.shape[-2]
    if out is None:
        alloc = torch.zeros if offsets is not None else torch.empty
        out = alloc(M, N // 2 if swiglu else N, dtype=x.dtype, device=x.device)
    if rope is not None and (offsets is not None or swiglu or N % 128):
        raise ValueError("gemm_tile: the RoPE epilogue is dense, without SwiGLU, N % 128 == 0")
    if rowscale is not None and (offsets is not None or not (swiglu or rope is not None)):
        raise ValueError("gemm_tile: the row scale is for the dense fused consumers (SwiGLU or RoPE)")
    if not _gpu(x):
        if packed:
            w = (torch.stack([unpack_skinny(e) for e in w]) if offsets is not None else unpack_skinny(w))
        inv = None
        if rowscale is not None:
            ssp, eps = rowscale
            inv = torch.rsqrt(ssp[:M].float().sum(1, keepdim=True) / x.shape[1] + eps)

        def one(xr, wr):
            y = torch.nn.functional.linear(xr.float(), wr.float())
            if inv is not None:
                y = y * inv
            y = y.to(x.dtype)
            if swiglu == 8:
                g = y.view(y.shape[0], -1, 16)
                return (torch.nn.functional.silu(g[..., :8].float()) * g[..., 8:].float()).reshape(y.shape[0], -1).to(x.dtype)
            return silu_mul(y, interleaved=True) if swiglu else y
        if offsets is None:
            out.copy_(one(x, w))
            if rope is not None:
                pos, cs, heads = rope
                h = out[:, : heads * 128].view(M, heads, 128).float()
                c = cs[pos.long(), :64].float()[:, None]
                s_ = cs[pos.long(), 64:].float()[:, None]
                a, b = h[..., :64], h[..., 64:]
                out[:, : heads * 128] = torch.cat([a * c - b * s_, b * c + a * s_], -1).reshape(M, -1).to(out.dtype)
        else:
            off = offsets.tolist()
            for e in range(w.shape[0]):
                a, b = off[e], off[e + 1]
                if b > a:
                    out[a:b] = one(x[a:b], w[e])
        return out
    rs_part, rs_eps = rowscale if rowscale is not None else (None, 1e-5)
    if rowscale is not None and algo != 1:
        raise ValueError("gemm_tile: the row scale needs schedule 1")
    if rope is not None:
        pos, cs, heads = rope
        native().gemm_tile(out, x.contiguous(), w, None, False, algo, pos, cs, heads, rs_part, rs_eps)
    elif rowscale is not None:
        native().gemm_tile(out, x.contiguous(), w, None, int(swiglu), algo, None, None, 0, rs_part, rs_eps)
    else:
        native().gemm_tile(out, x.contiguous(), w, offsets.contiguous() if offsets is not None else None,
                           int(swiglu), algo)
    return out


def gemm_tile_resid(x: torch.Tensor, w: torch.Tensor, resid: torch.Tensor, norm_w: torch.Tensor,
                    hw: Optional[torch.Tensor] = None, ss: Optional[torch.Tensor] = None) -> tuple:
    """A residual-producing prefill projection with the next RMSNorm's pass fused into its epilogue
    (csrc/gemm_tile.hip TILE_EPI_RESID; dense, N % 128 == 0): ``resid`` [M, N] <- bf16(resid +
    bf16(x @ w^T)) in place; returns ``(hw, ss)`` - hw = bf16(resid * norm_w) [M, N] and ss [M, N / 128]
    fp32 partial sums of resid^2 over each 128 columns, the operands of the consumer's row scale
    (``gemm_tile(hw, ..., rowscale=(ss, eps))`` = the projection of rms_norm(resid) * norm_w)."""
    M = x.shape[0]
    N = w.shape[0] * 16 if w.dim() == 4 else w.shape[0]  # row-major or fragment-packed W
    if N % 128 or resid.shape != (M, N):
        raise ValueError("gemm_tile_resid: N % 128 == 0 and resid [M, N]")
    hw = hw if hw is not None else torch.empty_like(resid)
    ss = ss if ss is not None else torch.empty(M, N // 128, dtype=torch.float32, device=resid.device)
    if not _gpu(x):
        if w.dim() == 4:
            w = unpack_skinny(w)
        y = torch.nn.functional.linear(x.float(), w.float()).to(x.dtype)
        h = (y.float() + resid.float()).to(resid.dtype)
        resid.copy_(h)
        hw.copy_((h.float() * norm_w.float()).to(hw.dtype))
        ss.copy_((h.float() ** 2).view(M, N // 128, 128).sum(2))
        return hw, ss
    native().gemm_tile(resid, x.contiguous(), w, None, False, TILE_ALGO, None, None, 0, None, 1e-5, resid, hw,
                       norm_w.contiguous(), ss)
    return hw, ss


# Prefill projections (qkv / o / gate_up + SwiGLU / down) on the hand-written 4-wave MFMA GEMM
# (csrc/gemm_tile.hip, two-barrier schedule) or hipBLASLt (torch F.linear).  The default ("tile")
# takes the tile kernel for every projection of at least TILE_MIN_M rows: in isolation hipBLASLt is
# 4-8 % faster on o / down (profiles/r03/gemm_ring_addressing.jsonl), but in the served headline
# the all-tile routing measured +1.4 % (three interleaved pairs, profiles/r04/bench_pg2_*.json:
# 25.06 vs 24.71 q/s), with qkv's RoPE fused into the tile epilogue.  "auto" = tile for the fused
# epilogues only (gate_up + SwiGLU, qkv + RoPE), hipBLASLt for o / down; "blas" = hipBLASLt for all.
# These routes apply to row-major weights; the ONE_LAYOUT models' fragment-packed weights (every
# Llama / Mixtral on the GPU) go to the tile kernel at any row count - hipBLASLt cannot read them.
# These are module constants (tools and tests set them for A/B runs), not environment switches.
PREFILL_GEMM = "tile"
QKV_ROPE_TILE = True  # qkv + fused RoPE on the tile kernel
# residual-add RMSNorm folded into the o / down epilogues and the qkv / gate_up row scale
FUSED_NORM = True
TILE_MIN_M = 1024  # below this a 256-row tile wastes most of its MFMAs on padding rows
# 1: the 4-wave kernel's two-barrier schedule, 0: one barrier per k-tile (K < 192 only)
TILE_ALGO = 1


def tile_shape_ok(M: int, N: int, K: int, swiglu: bool = False) -> bool:
    """gemm_tile takes this prefill GEMM (rows, output columns, depth)."""
    return (M >= TILE_MIN_M and N % 16 == 0 and K % 64 == 0 and K >= 128 and (not swiglu or N % 256 == 0)
            and N * K * 2 < (1 << 31))


def fused_norm_ok(M: int, d: int, n_qkv: int, n_o_in: int, n_13: int, f: int) -> bool:
    """The prefill layer may run with its RMSNorms folded into the tile GEMMs (gemm_tile_resid +
    row scale): every projection on the tile kernel (default routing), qkv with the RoPE epilogue,
    d a multiple of 128 with at most 64 partial sums per row (d <= 8192)."""
    return (FUSED_NORM and PREFILL_GEMM == "tile" and QKV_ROPE_TILE and d % 128 == 0 and d // 128 <= 64
            and n_qkv % 128 == 0 and tile_shape_ok(M, n_qkv, d) and tile_shape_ok(M, d, n_o_in)
            and tile_shape_ok(M, n_13, d, swiglu=True) and tile_shape_ok(M, d, f) and 256 * d * 2 < (1 << 31))


def w_out(w: torch.Tensor) -> int:
    """Output features of a dense projection weight: row-major [N, K] or fragment-packed
    [N/16, K/32, 64, 8] (pack_skinny)."""
    return w.shape[0] * 16 if w.dim() == 4 else w.shape[0]


def w_in(w: torch.Tensor) -> int:
    """Input features (K) of a row-major or fragment-packed dense projection weight."""
    return w.shape[1] * 32 if w.dim() == 4 else w.shape[1]


def prefill_linear(x: torch.Tensor, w: torch.Tensor, swiglu: bool = False,
                   out: Optional[torch.Tensor] = None, rope: Optional[tuple] = None,
                   rowscale: Optional[tuple] = None) -> torch.Tensor:
    """``x @ w^T`` for a prefill-sized ``x`` [M, K] and row-major ``w`` [N, K]; ``swiglu``: ``w`` is
    gate/up-interleaved (interleave_gate_up) and the result is silu(gate) * up [M, N / 2] - fused
    into the tile kernel's epilogue, or F.linear + silu_mul on the library path.
    ``rope = (positions, cos_sin, heads)`` (the qkv projection, head_dim 128): the tile kernel
    rotates heads 0 .. heads - 1 in its epilogue; returns ``(y, rotated)`` - rotated False when the
    library took the GEMM (the caller then applies RoPE itself).
    A fragment-packed ``w`` (pack_skinny, the ONE_LAYOUT resident form; ``swiglu=8`` with the
    interleave_gate_up8 pairing) always takes the tile kernel, whatever the row count - hipBLASLt
    cannot read it; on the CPU gemm_tile unpacks it for the fp32 reference."""
    M, K = x.shape
    if w.dim() == 4:
        if rope is not None:
            return gemm_tile(x, w, out=out, algo=TILE_ALGO, rope=rope, rowscale=rowscale), True
        return gemm_tile(x, w, swiglu=swiglu, out=out, algo=TILE_ALGO, rowscale=rowscale)
    N = w.shape[0]
    mode = PREFILL_GEMM
    tile_ok = _gpu(x) and tile_shape_ok(M, N, K, swiglu)
    if rope is not None:
        # the qkv projection takes the tile kernel whenever its RoPE epilogue applies: it replaces
        # rope_cache's read-rotate-write pass over q / k (more than the GEMM gives up to hipBLASLt)
        if (tile_ok and N % 128 == 0 and mode != "blas" and QKV_ROPE_TILE) or rowscale is not None:
            return gemm_tile(x, w, out=out, algo=TILE_ALGO, rope=rope, rowscale=rowscale), True
        return prefill_linear(x, w, out=out), False
    if rowscale is not None:  # the fused-norm consumer (the caller checked fused_norm_ok)
        return gemm_tile(x, w, swiglu=swiglu, out=out, algo=TILE_ALGO, rowscale=rowscale)
    use_tile = tile_ok and (mode == "tile" or (mode == "auto" and swiglu))
    if use_tile:
        return gemm_tile(x, w, swiglu=swiglu, out=out, algo=TILE_ALGO)
    y = torch.nn.functional.linear(x, w)
    if swiglu:
        return silu_mul(y, out=out, interleaved=True)
    return out.copy_(y) if out is not None else y


def moe_combine(y: torch.Tensor, inv_idx: torch.Tensor, w: torch.Tensor, T: int) -> torch.Tensor:
    if not _gpu(y):
        return ref.moe_combine(y, inv_idx, w, T)
    out = torch.empty(T, y.shape[1], dtype=y.dtype, device=y.device)
    native().moe_combine(out, y.contiguous(), inv_idx, w.contiguous())
    return out


def softmax_scale(head_dim: int) -> float:
    return 1.0 / math.sqrt(head_dim)
