"""Plain fp32 forward of a Llama-architecture CausalLM's own weights (no HIP kernels, no KV cache,
no fused epilogues): the numeric oracle for the GPU engine in ``__graft_entry__.smoke`` and the
real-shape GPU tests.  Weights are read from the model in their canonical row-major form (CausalLM.canonical: packed
or interleaved resident layouts undone), moved to
``device`` and upcast, so a GPU model can be checked against an fp32 pass on the CPU."""
from __future__ import annotations

from typing import Optional

import torch
import torch.nn.functional as F


@torch.no_grad()
def fp32_logits(model, ids: torch.Tensor, rows: Optional[list] = None, device: Optional[str] = None) -> torch.Tensor:
    """Logits [len(rows), vocab] of prompt ``ids`` (1-D) at positions ``rows`` (default: the last
    token), causal attention over the whole prompt.  TP=1 Llama arch (RoPE, RMSNorm, SwiGLU)."""
    c = model.cfg
    if c.arch != "llama" or c.is_moe or model.tp != 1:
        raise ValueError("fp32_logits: dense Llama-architecture models at TP=1")
    dev = torch.device(device) if device is not None else ids.device

    def w(t: torch.Tensor) -> torch.Tensor:
        return t.to(dev).float()

    ids = ids.to(dev).long()
    T = ids.numel()
    Hq, Hk, D = model.hq, model.hkv, model.D
    x = w(model.embed[ids.to(model.embed.device)])
    cs = w(model.cos_sin)
    pos = torch.arange(T, device=dev)
    cos, sin = cs[pos, : D // 2][:, None], cs[pos, D // 2:][:, None]

    def rope(t: torch.Tensor) -> torch.Tensor:
        a, b = t[..., : D // 2], t[..., D // 2:]
        return torch.cat([a * cos - b * sin, a * sin + b * cos], -1)

    for L in model.layers:
        h = F.rms_norm(x, (c.d_model,), w(L["attn_norm"]), c.norm_eps)
        q, k, v = (h @ w(model.canonical(L, "wqkv")).t()).split([Hq * D, Hk * D, Hk * D], 1)
        q, k = rope(q.view(T, Hq, D)), rope(k.view(T, Hk, D))
        att = F.scaled_dot_product_attention(q.transpose(0, 1)[None], k.transpose(0, 1)[None],
                                             v.view(T, Hk, D).transpose(0, 1)[None], is_causal=True,
                                             enable_gqa=Hq != Hk)[0]
        x = x + att.transpose(0, 1).reshape(T, Hq * D) @ w(model.canonical(L, "wo")).t()
        h = F.rms_norm(x, (c.d_model,), w(L["mlp_norm"]), c.norm_eps)
        gu = h @ w(model.canonical(L, "w13")).t()
        f = gu.shape[1] // 2
        x = x + (F.silu(gu[:, :f]) * gu[:, f:]) @ w(model.canonical(L, "w2")).t()
    rows = [T - 1] if rows is None else rows
    h = F.rms_norm(x[rows], (c.d_model,), w(model.final_norm), c.norm_eps)
    return (h @ w(model.canonical_head()).t())[:, : c.vocab_size]
