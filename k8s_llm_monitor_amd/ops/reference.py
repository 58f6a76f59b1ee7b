"""Plain-PyTorch fp32 references of every fused op.

They define the semantics the HIP kernels must reproduce (tests compare the two), and they
are the execution path for CPU tensors (unit tests, the GPT-2 CPU plumbing config).
KV-cache layouts (see ``csrc/rope_cache.hip``):

* ``k_cache`` ``[num_blocks, Hkv, D // 8, block_size, 8]``
* ``v_cache`` ``[num_blocks, Hkv, D, block_size]``, each block's tokens at positions ``v_perm(t)``
"""
from __future__ import annotations

import math

import torch
import torch.nn.functional as F


def rms_norm(x: torch.Tensor, w: torch.Tensor, eps: float) -> torch.Tensor:
    xf = x.float()
    y = xf * torch.rsqrt(xf.pow(2).mean(-1, keepdim=True) + eps) * w.float()
    return y.to(x.dtype)


def fused_add_rms_norm(x: torch.Tensor, residual: torch.Tensor, w: torch.Tensor, eps: float):
    s = (x.float() + residual.float()).to(x.dtype)
    return rms_norm(s, w, eps), s


def layer_norm(x, w, b, eps):
    return F.layer_norm(x.float(), (x.shape[-1],), w.float(), b.float(), eps).to(x.dtype)


def silu_mul(x: torch.Tensor, interleaved: bool = False) -> torch.Tensor:
    """silu(gate) * up; ``interleaved``: columns are [64 gate | 64 up] per 128."""
    f = x.shape[-1] // 2
    xf = x.float()
    if interleaved:
        t = xf.reshape(*xf.shape[:-1], f // 64, 2, 64)
        return (F.silu(t[..., 0, :]) * t[..., 1, :]).reshape(*xf.shape[:-1], f).to(x.dtype)
    return (F.silu(xf[..., :f]) * xf[..., f:]).to(x.dtype)


def gelu_tanh(x: torch.Tensor) -> torch.Tensor:
    return F.gelu(x.float(), approximate="tanh").to(x.dtype)


def embedding(ids: torch.Tensor, weight: torch.Tensor, vocab_start: int = 0) -> torch.Tensor:
    local = ids.long() - vocab_start
    ok = (local >= 0) & (local < weight.shape[0])
    out = weight[local.clamp(0, weight.shape[0] - 1)]
    return out * ok.unsqueeze(-1).to(out.dtype)


def rope_cos_sin(max_pos: int, head_dim: int, theta: float, scaling: dict | None = None,
                 device=None) -> torch.Tensor:
    """[max_pos, head_dim] fp32 table: first half cos, second half sin (neox pairing).

    ``scaling`` supports the Llama-3.1 ``{"rope_type": "llama3", "factor", "low_freq_factor",
    "high_freq_factor", "original_max_position_embeddings"}`` frequency remap.
    """
    half = head_dim // 2
    inv = 1.0 / (theta ** (torch.arange(0, half, dtype=torch.float64) * 2 / head_dim))
    if scaling and scaling.get("rope_type", scaling.get("type")) == "llama3":
        factor = scaling["factor"]
        lo, hi = scaling["low_freq_factor"], scaling["high_freq_factor"]
        orig = scaling["original_max_position_embeddings"]
        wavelen = 2 * math.pi / inv
        lo_wl, hi_wl = orig / lo, orig / hi
        smooth = (orig / wavelen - lo) / (hi - lo)
        scaled = torch.where(wavelen > lo_wl, inv / factor, inv)
        mid = (wavelen <= lo_wl) & (wavelen >= hi_wl)
        inv = torch.where(mid, (1 - smooth) * inv / factor + smooth * inv, scaled)
    t = torch.arange(max_pos, dtype=torch.float64)
    ang = torch.outer(t, inv)
    return torch.cat([ang.cos(), ang.sin()], dim=-1).float().to(device)


def apply_rope(x: torch.Tensor, positions: torch.Tensor, cos_sin: torch.Tensor) -> torch.Tensor:
    """x: [T, H, D]; returns rotated fp32."""
    d = x.shape[-1]
    half = d // 2
    cs = cos_sin[positions.long()]
    c, s = cs[:, None, :half], cs[:, None, half:]
    xf = x.float()
    x1, x2 = xf[..., :half], xf[..., half:]
    return torch.cat([x1 * c - x2 * s, x2 * c + x1 * s], dim=-1)


def rope_and_cache(qkv, positions, cos_sin, k_cache, v_cache, slot_mapping, Hq, Hkv, D, apply_rope_=True):
    T = qkv.shape[0]
    q = qkv[:, : Hq * D].view(T, Hq, D)
    k = qkv[:, Hq * D:(Hq + Hkv) * D].view(T, Hkv, D)
    v = qkv[:, (Hq + Hkv) * D:(Hq + 2 * Hkv) * D].view(T, Hkv, D)
    if apply_rope_:
        q.copy_(apply_rope(q, positions, cos_sin).to(qkv.dtype))
        k.copy_(apply_rope(k, positions, cos_sin).to(qkv.dtype))
    if slot_mapping is not None and slot_mapping.numel() > 0:
        write_kv_cache(k, v, k_cache, v_cache, slot_mapping)


def v_perm(t):
    """V-cache position of block token t (common.h v_perm): bits 2 and 3 swapped, an involution."""
    return (t & ~12) | ((t & 4) << 1) | ((t & 8) >> 1)


def write_kv_cache(k, v, k_cache, v_cache, slot_mapping):
    bs = k_cache.shape[3]
    D = v_cache.shape[2]
    sm = slot_mapping.long()
    ok = sm >= 0
    sm, k, v = sm[ok], k[ok], v[ok]
    blk, off = sm // bs, sm % bs
    kk = k.view(k.shape[0], k.shape[1], D // 8, 8)
    k_cache[blk, :, :, off, :] = kk
    v_cache[blk, :, :, v_perm(off)] = v


def gather_kv(k_cache, v_cache, block_table: torch.Tensor, seq_len: int):
    """Contiguous [L, Hkv, D] keys and values of one sequence."""
    bs = k_cache.shape[3]
    nb = (seq_len + bs - 1) // bs
    blocks = block_table[:nb].long()
    kb = k_cache[blocks]  # [nb, Hkv, D/8, bs, 8]
    nbk, hkv, p, _, _ = kb.shape
    k = kb.permute(0, 3, 1, 2, 4).reshape(nbk * bs, hkv, p * 8)[:seq_len]
    vb = v_cache[blocks]  # [nb, Hkv, D, bs], tokens at positions v_perm(t)
    vb = vb[..., v_perm(torch.arange(bs, device=vb.device))]
    v = vb.permute(0, 3, 1, 2).reshape(nbk * bs, hkv, -1)[:seq_len]
    return k, v


def attention(q, k, v, scale: float, causal: bool) -> torch.Tensor:
    """q [Tq, Hq, D], k/v [Tk, Hkv, D] (GQA broadcast); fp32 result [Tq, Hq, D].
    causal aligns the last query with the last key."""
    hq, hkv = q.shape[1], k.shape[1]
    g = hq // hkv
    qf = q.float().transpose(0, 1)
    kf = k.float().repeat_interleave(g, dim=1).transpose(0, 1)
    vf = v.float().repeat_interleave(g, dim=1).transpose(0, 1)
    s = qf @ kf.transpose(1, 2) * scale
    if causal:
        tq, tk = q.shape[0], k.shape[0]
        mask = torch.ones(tq, tk, dtype=torch.bool, device=q.device).tril(tk - tq)
        s = s.masked_fill(~mask, float("-inf"))
    p = torch.softmax(s, dim=-1)
    return (p @ vf).transpose(0, 1)


def paged_decode(q, k_cache, v_cache, block_tables, seq_lens, Hq, Hkv, D, scale):
    """q [B, >=Hq*D]; returns [B, Hq*D] in q.dtype."""
    B = seq_lens.shape[0]
    out = torch.zeros(B, Hq * D, dtype=q.dtype, device=q.device)
    for b in range(B):
        L = int(seq_lens[b])
        if L <= 0:
            continue
        k, v = gather_kv(k_cache, v_cache, block_tables[b], L)
        qb = q[b, : Hq * D].view(1, Hq, D)
        out[b] = attention(qb, k, v, scale, causal=False).reshape(-1).to(q.dtype)
    return out


def flash_prefill(qkv, cu_seqlens, Hq, Hkv, D, scale):
    T = qkv.shape[0]
    out = torch.empty(T, Hq * D, dtype=qkv.dtype, device=qkv.device)
    cu = cu_seqlens.tolist()
    for i in range(len(cu) - 1):
        a, b = cu[i], cu[i + 1]
        if b <= a:
            continue
        x = qkv[a:b]
        q = x[:, : Hq * D].view(b - a, Hq, D)
        k = x[:, Hq * D:(Hq + Hkv) * D].view(b - a, Hkv, D)
        v = x[:, (Hq + Hkv) * D:(Hq + 2 * Hkv) * D].view(b - a, Hkv, D)
        out[a:b] = attention(q, k, v, scale, causal=True).reshape(b - a, -1).to(qkv.dtype)
    return out


def paged_prefill(qkv, cu_seqlens, ctx_start, k_cache, v_cache, block_tables, Hq, Hkv, D, scale):
    """Queries = each sequence's new rows of ``qkv``; keys/values = positions [0, ctx_start + new)
    from the paged cache (which already holds the new tokens)."""
    T = qkv.shape[0]
    out = torch.empty(T, Hq * D, dtype=qkv.dtype, device=qkv.device)
    cu, cs = cu_seqlens.tolist(), ctx_start.tolist()
    for i in range(len(cu) - 1):
        a, b = cu[i], cu[i + 1]
        if b <= a:
            continue
        k, v = gather_kv(k_cache, v_cache, block_tables[i], cs[i] + b - a)
        q = qkv[a:b, : Hq * D].view(b - a, Hq, D)
        out[a:b] = attention(q, k, v, scale, causal=True).reshape(b - a, -1).to(qkv.dtype)
    return out


def greedy(logits: torch.Tensor) -> torch.Tensor:
    return logits.float().argmax(-1).to(torch.int32)


def moe_route(logits: torch.Tensor, k: int, renorm: bool):
    p = torch.softmax(logits.float(), dim=-1)
    w, ids = torch.topk(p, k, dim=-1)
    if renorm:
        w = w / w.sum(-1, keepdim=True)
    return ids.to(torch.int32), w


def moe_align(ids: torch.Tensor, E: int):
    flat = ids.reshape(-1).long()
    order = torch.argsort(flat, stable=True)
    counts = torch.bincount(flat, minlength=E)
    offsets = torch.zeros(E + 1, dtype=torch.int32, device=ids.device)
    offsets[1:] = torch.cumsum(counts, 0).to(torch.int32)
    inv = torch.empty_like(order)
    inv[order] = torch.arange(order.numel(), device=ids.device)
    return offsets, order.to(torch.int32), inv.to(torch.int32)


def moe_combine(y: torch.Tensor, inv_idx: torch.Tensor, w: torch.Tensor, T: int) -> torch.Tensor:
    K = w.shape[1]
    g = y.float()[inv_idx.long()].view(T, K, -1)
    return (g * w.float().unsqueeze(-1)).sum(1).to(y.dtype)
