"""Batched attention for the CPU serving path (config 1: GPT-2-small plumbing, SURVEY.md §2.12
K-11 - torch ops are allowed there).

:mod:`.reference` stays the fp32 test oracle for the HIP kernels; it gathers each sequence's keys
separately and expands GQA with ``repeat_interleave``, which made the CPU decode step loop over the
batch in Python (VERDICT r5 Weak #5).  Here one decode step does ONE block-table gather for the
whole batch and two einsums in the cache's own layouts (paged_decode); prefill runs one
``scaled_dot_product_attention`` per sequence over its gathered cache span (fp32).

Cache layouts are the engine's (common.h): K [blocks, Hkv, D/8, bs, 8], V [blocks, Hkv, D, bs]
with token t of a block stored at position v_perm(t).
"""
from __future__ import annotations

import torch
import torch.nn.functional as F

from .reference import v_perm

_VPERM: dict = {}


def _vperm_index(bs: int, device: torch.device) -> torch.Tensor:
    key = (bs, str(device))
    t = _VPERM.get(key)
    if t is None:
        t = _VPERM[key] = v_perm(torch.arange(bs, device=device))
    return t


def gather_batch(k_cache: torch.Tensor, v_cache: torch.Tensor, block_tables: torch.Tensor, nb: int):
    """Keys / values of the first ``nb`` blocks of every row of ``block_tables`` [B, >= nb]:
    fp32 [B, Hkv, nb * bs, D] each, tokens in sequence order (entries < 0 read block 0; mask them)."""
    bt = block_tables[:, :nb].long().clamp(min=0)
    kb = k_cache[bt]  # [B, nb, Hkv, D/8, bs, 8]
    B, _, hkv, p, bs, _ = kb.shape
    k = kb.permute(0, 2, 1, 4, 3, 5).reshape(B, hkv, nb * bs, p * 8).float()
    vb = v_cache[bt].index_select(-1, _vperm_index(bs, v_cache.device))  # [B, nb, Hkv, D, bs]
    v = vb.permute(0, 2, 1, 4, 3).reshape(B, hkv, nb * bs, -1).float()
    return k, v


def paged_decode(q: torch.Tensor, k_cache: torch.Tensor, v_cache: torch.Tensor, block_tables: torch.Tensor,
                 seq_lens: torch.Tensor, Hq: int, Hkv: int, D: int, scale: float) -> torch.Tensor:
    """One query row per sequence (q [B, >= Hq*D]) over its paged cache; [B, Hq*D] in q.dtype.

    The blocks are gathered once for the whole batch and used in the cache's own layouts (no
    transposing copy): scores by one einsum over K [B, nb, Hkv, D/8, bs, 8] (GQA as a group axis),
    softmax in fp32 over the ragged lengths, the probabilities permuted to V's in-block token order
    (v_perm) - a [B, Hq, L] shuffle instead of one over V - and one einsum against V
    [B, nb, Hkv, D, bs].  Operands stay in the cache dtype (bf16: the CPU's bf16 matrix units,
    fp32 accumulation; P rounded to bf16 as the GPU kernel's PV MFMA does)."""
    B = seq_lens.shape[0]
    out = torch.zeros(B, Hq * D, dtype=q.dtype, device=q.device)
    if B == 0:
        return out
    lens = seq_lens.long()
    lmax = int(lens.max())
    if lmax <= 0:
        return out
    bs = k_cache.shape[3]
    nb = (lmax + bs - 1) // bs
    bt = block_tables[:, :nb].long().clamp(min=0)
    kb, vb = k_cache[bt], v_cache[bt]  # [B, nb, Hkv, D/8, bs, 8], [B, nb, Hkv, D, bs]
    G = Hq // Hkv
    qv = q[:, : Hq * D].reshape(B, Hkv, G, D // 8, 8).to(kb.dtype)
    s = torch.einsum("bhgpe,bnhpte->bhgnt", qv, kb).float().reshape(B, Hkv, G, nb * bs) * scale
    pos = torch.arange(nb * bs, device=q.device)
    s = s.masked_fill((pos[None, :] >= lens[:, None]).view(B, 1, 1, nb * bs), float("-inf"))
    p = torch.softmax(s, dim=-1).view(B, Hkv, G, nb, bs).index_select(-1, _vperm_index(bs, q.device))
    o = torch.einsum("bhgnt,bnhdt->bhgd", p.to(vb.dtype), vb)
    live = lens > 0
    out[live] = o.reshape(B, Hq * D)[live].to(q.dtype)
    return out


def _causal(q: torch.Tensor, k: torch.Tensor, v: torch.Tensor, scale: float, Hq: int, Hkv: int) -> torch.Tensor:
    """q [Tq, Hq, D] against k / v [Hkv, Tk, D] (fp32), the last query aligned with the last key."""
    tq, tk = q.shape[0], k.shape[1]
    qf = q.float().transpose(0, 1).unsqueeze(0)
    if tq == tk:
        o = F.scaled_dot_product_attention(qf, k.unsqueeze(0), v.unsqueeze(0), is_causal=True, scale=scale,
                                           enable_gqa=Hq != Hkv)
    else:
        mask = torch.ones(tq, tk, dtype=torch.bool, device=q.device).tril(tk - tq)
        o = F.scaled_dot_product_attention(qf, k.unsqueeze(0), v.unsqueeze(0), attn_mask=mask, scale=scale,
                                           enable_gqa=Hq != Hkv)
    return o[0].transpose(0, 1)


def flash_prefill(qkv: torch.Tensor, cu_seqlens: torch.Tensor, Hq: int, Hkv: int, D: int, scale: float) -> torch.Tensor:
    """Causal attention of each sequence's rows of the fused qkv projection."""
    T = qkv.shape[0]
    out = torch.empty(T, Hq * D, dtype=qkv.dtype, device=qkv.device)
    cu = cu_seqlens.tolist()
    for i in range(len(cu) - 1):
        a, b = cu[i], cu[i + 1]
        if b <= a:
            continue
        x = qkv[a:b]
        q = x[:, : Hq * D].view(b - a, Hq, D)
        k = x[:, Hq * D:(Hq + Hkv) * D].view(b - a, Hkv, D).float().transpose(0, 1)
        v = x[:, (Hq + Hkv) * D:(Hq + 2 * Hkv) * D].view(b - a, Hkv, D).float().transpose(0, 1)
        out[a:b] = _causal(q, k, v, scale, Hq, Hkv).reshape(b - a, -1).to(qkv.dtype)
    return out


def paged_prefill(qkv: torch.Tensor, cu_seqlens: torch.Tensor, ctx_start: torch.Tensor, k_cache: torch.Tensor,
                  v_cache: torch.Tensor, block_tables: torch.Tensor, Hq: int, Hkv: int, D: int,
                  scale: float) -> torch.Tensor:
    """Each sequence's new rows (positions ctx_start ..) against its cached prefix + new tokens."""
    T = qkv.shape[0]
    out = torch.empty(T, Hq * D, dtype=qkv.dtype, device=qkv.device)
    cu, cs = cu_seqlens.tolist(), ctx_start.tolist()
    bs = k_cache.shape[3]
    for i in range(len(cu) - 1):
        a, b = cu[i], cu[i + 1]
        if b <= a:
            continue
        L = cs[i] + b - a
        k, v = gather_batch(k_cache, v_cache, block_tables[i:i + 1], (L + bs - 1) // bs)
        q = qkv[a:b, : Hq * D].view(b - a, Hq, D)
        out[a:b] = _causal(q, k[0, :, :L], v[0, :, :L], scale, Hq, Hkv).reshape(b - a, -1).to(qkv.dtype)
    return out
