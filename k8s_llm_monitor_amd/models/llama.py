"""Decoder-only causal LMs served by the diagnostic engine: Llama-3 (dense), Mixtral (MoE) and
GPT-2 (the CPU plumbing config), with Megatron tensor parallelism.

Nothing here exists in the reference ("no LLM, no GPU code"); the model replaces
the remote ``callLLMAPI`` step of the doc sketch ``docs/metrics-usage-example.md:244-306``.

Prefill layer (GPU, >= 1024 rows, TP=1; ``_prefill_fused_norm``), every GEMM on the hand-written
256 x 256 MFMA tile kernel (ops/csrc/gemm_tile.hip) with its epilogue doing the elementwise work:

  qkv (+ RoPE of q / k, rows scaled by 1/rms) -> rope_and_cache (paged KV write) -> flash_prefill
  -> o (+ residual add, next norm's operand and sums of squares) -> gate_up (+ SwiGLU, row scale)
  -> down (+ residual add, ...)

TP > 1 prefill runs as two micro-batches whose row-parallel all-reduces overlap each other's
compute (``_prefill_overlap``).

Decode layer (``_decode_layers_skinny``, 7 launches inside one hipGraph): qkv (split-K slabs) ->
paged_decode_fused (slab reduce + RoPE + KV write + attention) -> o (slabs) -> add_norm_partial
(residual add, deferred norm) -> gate_up + SwiGLU -> down (slabs) -> add_norm_partial.  Dense
models whose weights fit a quarter of the device run the projections and the LM head on the
shared-A decode GEMM over decode-only fragment-packed copies (ops/csrc/gemm_decode.hip); larger
ones (70B at TP=1) on the row-major skinny kernel over the prefill tensors (gemm_skinny.hip).

Weights are stored fused and pre-sharded: ``wqkv`` [(Hq+2Hkv)/tp * D, d] (column-parallel),
``wo`` [d, Hq/tp * D] (row-parallel), ``w13`` [2F/tp, d] (this rank's gate and up rows, stored
interleaved per 128 rows as [64 gate | 64 up] - see _init_skinny), ``w2`` [d, F/tp].  Random init is seeded per tensor name, and every rank generates the
full tensor then keeps its shard, so any TP degree reproduces the TP=1 model exactly.
"""
from __future__ import annotations

import hashlib
import math
import os
from dataclasses import dataclass
from typing import Optional

import torch
import torch.nn.functional as F

from .. import ops
from ..ops import reference as ref
from ..parallel.comm import (kv_head_range, shard_range, tp_all_gather_last, tp_all_gather_rows, tp_all_reduce,
                             tp_all_reduce_async, tp_all_to_all)
from ..parallel.state import ParallelState, get_state
from .config import ModelConfig


@dataclass
class AttnMeta:
    """Per-step batch metadata (built by the engine's model runner)."""

    is_prefill: bool
    positions: torch.Tensor  # [T] int32
    slot_mapping: torch.Tensor  # [T] int32, -1 = do not write the cache
    # prefill (whole prompts in this step)
    cu_seqlens: Optional[torch.Tensor] = None  # [S+1] int32
    qb_seq: Optional[torch.Tensor] = None  # flash_prefill q-block schedule
    qb_start: Optional[torch.Tensor] = None
    logits_idx: Optional[torch.Tensor] = None  # [S] int64 rows that produce logits
    ctx_start: Optional[torch.Tensor] = None  # [S] int32 cached prefix tokens (paged prefill) or None
    # decode (one token per sequence)
    block_tables: Optional[torch.Tensor] = None  # [B, W] int32
    seq_lens: Optional[torch.Tensor] = None  # [B] int32 (including the token being decoded)
    decode_ws: Optional[tuple] = None  # paged_decode partial buffers
    # mixed prefill+decode step (is_prefill): the first num_decode rows are single decode tokens
    # attending their paged context through paged_decode; cu_seqlens / qb_* / ctx_start /
    # block_tables then describe the prefill rows that follow
    num_decode: int = 0
    dec_block_tables: Optional[torch.Tensor] = None  # [num_decode, W] int32
    dec_seq_lens: Optional[torch.Tensor] = None  # [num_decode] int32 (including the decoded token)
    # pipelined decode inputs: row i feeds dec_prev[dec_src[i]] when dec_src[i] >= 0 (the token the
    # previous step sampled, still on the device), else ids[i]; resolved inside the first kernel
    dec_src: Optional[torch.Tensor] = None  # [B] int32
    dec_prev: Optional[torch.Tensor] = None  # [>= B] int32
    # TP > 1 prefill as two micro-batches of whole sequences: (meta of rows [0, TA), meta of rows
    # [TA, T), TA); their row-parallel all-reduces overlap each other's compute (_prefill_overlap)
    micro: Optional[tuple] = None


def _seed_for(name: str, seed: int) -> int:
    h = hashlib.blake2b(f"{seed}:{name}".encode(), digest_size=8).digest()
    return int.from_bytes(h, "little") & 0x7FFF_FFFF_FFFF_FFFF


class CausalLM:
    # path selection for tests and tools (class attributes, not environment switches):
    # SKINNY_DECODE False = decode through the plain row-major path (the fp32-reference form of the
    # real-shape tests); DECODE_GEMM "auto" | "dec" | "rm" = the decode projections' kernel (_want_dec)
    SKINNY_DECODE = True
    DECODE_GEMM = "auto"
    # ONE resident copy of every dense Llama projection on the GPU: the decode GEMMs' fragment-packed
    # layout, which the prefill tile GEMM reads as well (gemm_tile wpk mode - bit-identical to the
    # row-major form and within +-1.4 % of its speed: profiles/r06/gemm_packed_w_*.jsonl); the
    # row-major tensors are dropped.  "force": also on the CPU (tests).
    ONE_LAYOUT = True

    def __init__(self, cfg: ModelConfig, device: torch.device | str = "cpu", dtype=torch.bfloat16, seed: int = 0,
                 pstate: Optional[ParallelState] = None, init_std: float = 0.02, init: str = "random"):
        """``init``: "random" (seeded per tensor name) or "empty" (uninitialised storage, for
        models about to be filled by models/checkpoint.load_checkpoint)."""
        if init not in ("random", "empty"):
            raise ValueError(f"init must be 'random' or 'empty', not {init!r}")
        self._empty_init = init == "empty"
        self.cfg = cfg
        self.device = torch.device(device)
        self.dtype = dtype
        self.seed = seed
        self.ps = pstate or get_state()
        tp, r = self.ps.tp_size, self.ps.tp_rank
        kv_ok = cfg.n_kv_heads % tp == 0 or tp % cfg.n_kv_heads == 0  # shard, or replicate (kv_head_range)
        if cfg.n_heads % tp or not kv_ok or cfg.ffn_dim % tp or cfg.vocab_size_padded(tp) % tp:
            raise ValueError(f"{cfg.name}: heads/ffn/vocab not divisible by tp={tp}")
        self.tp, self.rank = tp, r
        self.hq = cfg.n_heads // tp
        self.hkv = max(1, cfg.n_kv_heads // tp)
        self.D = cfg.head_dim
        self.f_local = cfg.ffn_dim // tp
        self.vocab_padded = cfg.vocab_size_padded(tp)
        self.v_lo, self.v_hi = shard_range(self.vocab_padded, tp, r)
        self.scale = 1.0 / math.sqrt(self.D)
        self.std = init_std
        if cfg.is_moe:
            if cfg.n_experts % tp:
                raise ValueError("n_experts must be divisible by tp for expert parallelism")
            self.e_lo, self.e_hi = shard_range(cfg.n_experts, tp, r)
        self.moe_comm = os.environ.get("K8SLLM_MOE_COMM", "a2a")  # "a2a" (prefill all-to-all EP) | "allreduce"
        # MoE prefill GEMMs: "grouped" (default) = one launch per projection over all local
        # experts from the device-side offsets (gemm_tile.hip 256 x 256 tiles, SwiGLU fused; zero
        # host syncs, capturable); "loop" = one hipBLASLt GEMM per expert after a host sync of the
        # expert offsets.  Mixtral-8x7B end to end: 8.14 vs 8.11 q/s (profiles/r02)
        self._moe_grouped = True
        # MoE decode at TP>1: "allreduce" = every rank runs its experts on every (replicated)
        # token, dense-masked, then one all-reduce; "a2a" = expert-parallel dispatch / combine with
        # static-capacity all-to-alls (_moe_a2a_decode, graph-capturable)
        self.moe_decode = os.environ.get("K8SLLM_MOE_DECODE", "allreduce")
        self.layers: list[dict] = []
        self._w13_il = False  # w13 gate/up-interleaved per 128 rows (set by _init_skinny)
        self._packed = False  # ONE_LAYOUT: the dense projections are resident fragment-packed only
        self._swg = True  # gemm_tile's SwiGLU pairing of w13: True = per 128 rows, 8 = per 16 (packed)
        self.skinny_layout = None
        self._build()
        self._init_skinny()
        self.cos_sin = None
        if cfg.arch == "llama":
            self.cos_sin = ref.rope_cos_sin(cfg.max_position, self.D, cfg.rope_theta, cfg.rope_scaling,
                                            device=self.device)

    # ------------------------------------------------------------------ weights
    def _rand(self, name: str, shape, std: Optional[float] = None) -> torch.Tensor:
        if self._empty_init:
            return torch.empty(shape, dtype=self.dtype, device=self.device)
        g = torch.Generator(device=self.device)
        g.manual_seed(_seed_for(name, self.seed))
        t = torch.empty(shape, dtype=torch.float32 if self.device.type == "cpu" else self.dtype, device=self.device)
        t.normal_(0.0, self.std if std is None else std, generator=g)
        return t.to(self.dtype)

    def _ones(self, n) -> torch.Tensor:
        return torch.ones(n, dtype=self.dtype, device=self.device)

    def _zeros(self, n) -> torch.Tensor:
        return torch.zeros(n, dtype=self.dtype, device=self.device)

    def _build(self) -> None:
        c = self.cfg
        d, D, tp, r = c.d_model, self.D, self.tp, self.rank
        out_std = self.std / math.sqrt(2 * c.n_layers)
        emb = self._rand("embed", (self.vocab_padded, d))
        self.embed = emb[self.v_lo:self.v_hi].contiguous()
        del emb
        if c.tie_embeddings:
            self.lm_head = self.embed
        else:
            lm = self._rand("lm_head", (self.vocab_padded, d))
            self.lm_head = lm[self.v_lo:self.v_hi].contiguous()
            del lm
        if c.arch == "gpt2":
            self.pos_embed = self._rand("pos_embed", (c.max_position, d), 0.01)
            self.final_norm = (self._ones(d), self._zeros(d))
        else:
            self.final_norm = self._ones(d)
        q_lo, q_hi = shard_range(c.n_heads * D, tp, r)
        kv_lo, kv_hi = kv_head_range(c.n_kv_heads, D, tp, r)
        f_lo, f_hi = shard_range(c.ffn_dim, tp, r)
        for i in range(c.n_layers):
            p = f"layers.{i}."
            L: dict = {}
            wq = self._rand(p + "wq", (c.n_heads * D, d))
            wk = self._rand(p + "wk", (c.n_kv_heads * D, d))
            wv = self._rand(p + "wv", (c.n_kv_heads * D, d))
            L["wqkv"] = torch.cat([wq[q_lo:q_hi], wk[kv_lo:kv_hi], wv[kv_lo:kv_hi]], 0).contiguous()
            del wq, wk, wv
            wo = self._rand(p + "wo", (d, c.n_heads * D), out_std)
            L["wo"] = wo[:, q_lo:q_hi].contiguous()
            del wo
            if c.arch == "gpt2":
                L["ln1"] = (self._ones(d), self._zeros(d))
                L["ln2"] = (self._ones(d), self._zeros(d))
                bqkv = self._rand(p + "bqkv", ((c.n_heads + 2 * c.n_kv_heads) * D,), 0.01)
                nq, nk = c.n_heads * D, c.n_kv_heads * D
                L["bqkv"] = torch.cat([bqkv[q_lo:q_hi], bqkv[nq + kv_lo:nq + kv_hi],
                                       bqkv[nq + nk + kv_lo:nq + nk + kv_hi]]).contiguous()
                L["bo"] = self._rand(p + "bo", (d,), 0.01)  # added once (rank 0 adds it before the reduce)
                w1 = self._rand(p + "w1", (c.ffn_dim, d))
                L["w1"] = w1[f_lo:f_hi].contiguous()
                L["b1"] = self._rand(p + "b1", (c.ffn_dim,), 0.01)[f_lo:f_hi].contiguous()
                w2 = self._rand(p + "w2", (d, c.ffn_dim), out_std)
                L["w2"] = w2[:, f_lo:f_hi].contiguous()
                L["b2"] = self._rand(p + "b2", (d,), 0.01)
                del w1, w2
            else:
                L["attn_norm"] = self._ones(d)
                L["mlp_norm"] = self._ones(d)
                if c.is_moe:
                    L["router"] = self._rand(p + "router", (c.n_experts, d))
                    w13, w2s = [], []
                    for e in range(self.e_lo, self.e_hi):
                        g = self._rand(p + f"experts.{e}.w1", (c.ffn_dim, d))
                        u = self._rand(p + f"experts.{e}.w3", (c.ffn_dim, d))
                        w13.append(torch.cat([g, u], 0))
                        w2s.append(self._rand(p + f"experts.{e}.w2", (d, c.ffn_dim), out_std))
                        del g, u
                    L["w13"] = torch.stack(w13).contiguous()  # [E_local, 2F, d]
                    L["w2"] = torch.stack(w2s).contiguous()  # [E_local, d, F]
                    del w13, w2s
                else:
                    g = self._rand(p + "w1", (c.ffn_dim, d))
                    u = self._rand(p + "w3", (c.ffn_dim, d))
                    L["w13"] = torch.cat([g[f_lo:f_hi], u[f_lo:f_hi]], 0).contiguous()
                    del g, u
                    w2 = self._rand(p + "w2", (d, c.ffn_dim), out_std)
                    L["w2"] = w2[:, f_lo:f_hi].contiguous()
                    del w2
            self.layers.append(L)

    def resident_weight_bytes(self) -> int:
        """Bytes of every distinct weight tensor this rank holds (parameters, decode-layout copies
        and the LM head's packed copy; a tensor referenced under two keys counts once)."""
        seen, n = set(), 0
        ts = [self.embed, self.lm_head, getattr(self, "lm_head_d", None), self.final_norm]
        for L in self.layers:
            for v in L.values():
                ts.extend(v if isinstance(v, tuple) else (v,))
        for t in ts:
            if isinstance(t, torch.Tensor) and t.data_ptr() not in seen:
                seen.add(t.data_ptr())
                n += t.numel() * t.element_size()
        return n

    def num_local_params(self) -> int:
        n = self.embed.numel() + (0 if self.cfg.tie_embeddings else self.lm_head.numel())
        for L in self.layers:
            for k, v in L.items():
                if k.endswith(("_p", "_d", "_pg", "_dg")):  # decode-layout copies (_init_skinny) are not parameters
                    continue
                if isinstance(v, tuple):
                    n += sum(t.numel() for t in v)
                else:
                    n += v.numel()
        return n

    # ------------------------------------------------------------------ forward
    def embed_tokens(self, ids: torch.Tensor) -> torch.Tensor:
        if self.tp == 1:
            if ids.is_cuda:
                return ops.embedding(ids, self.embed)
            return self.embed[ids.long()]
        x = ops.embedding(ids, self.embed, vocab_start=self.v_lo)
        return tp_all_reduce(x, self.ps)

    def _attention(self, L: dict, x: torch.Tensor, meta: AttnMeta, kv) -> torch.Tensor:
        o = self._attn_core(L, x, meta, kv)
        y = ops.prefill_linear(o, L["wo"]) if "bo" not in L else F.linear(o, L["wo"])
        if "bo" in L and self.rank == 0:
            y += L["bo"]
        return tp_all_reduce(y, self.ps)

    def _attn_core(self, L: dict, x: Optional[torch.Tensor], meta: AttnMeta, kv, slabs: Optional[tuple] = None,
                   rows: Optional[int] = None, rownorm: Optional[tuple] = None,
                   rowscale: Optional[tuple] = None) -> torch.Tensor:
        """QKV projection, RoPE + KV-cache write, attention; returns the per-head output [T, Hq*D].
        ``slabs = (workspace, splits)``: decode QKV by the split-K skinny GEMM over ``x`` (row-major
        or fragment-packed with ``rows`` valid rows), reduced inside rope_and_cache; the attention
        output is then written fragment-packed for the o_proj skinny GEMM."""
        c = self.cfg
        k_cache, v_cache = kv if kv is not None else (None, None)
        partial, ns = None, 0
        roped = False  # q / k already rotated by the qkv GEMM's epilogue
        T = rows if rows is not None else x.shape[0]
        cs = self.cos_sin if self.cos_sin is not None else _dummy_cs(self)
        if slabs is not None:
            ws, splits = slabs
            ns = self._proj_slabs(L, "wqkv", x, T, splits, rownorm)
            if self._attn_rope and not meta.is_prefill and k_cache is not None and c.arch == "llama":
                # the attention kernel reduces the slabs, applies RoPE and writes the new k / v
                out = ops.packed_empty(T, self.hq * self.D, self.dtype, self.device)
                return ops.paged_decode_fused(ws, ns, meta.positions, cs, meta.slot_mapping, k_cache, v_cache,
                                              meta.block_tables, meta.seq_lens, self.hq, self.hkv, self.D, self.scale,
                                              workspace=meta.decode_ws, out=out)
            partial = ws
            qkv = torch.empty(T, ops.w_out(L["wqkv"]), dtype=self.dtype, device=self.device)
        elif "bqkv" in L:
            qkv = F.linear(x, L["wqkv"], L["bqkv"])
        elif c.arch == "llama" and self.D == 128 and self.cos_sin is not None:
            # prefill-sized qkv on the tile kernel: RoPE of q / k fused into its epilogue
            qkv, roped = ops.prefill_linear(x, L["wqkv"], rope=(meta.positions, cs, self.hq + self.hkv),
                                            rowscale=rowscale)
        else:
            qkv = ops.prefill_linear(x, L["wqkv"])
        ops.rope_and_cache(qkv, meta.positions, cs, k_cache, v_cache,
                           meta.slot_mapping if k_cache is not None else None, self.hq, self.hkv, self.D,
                           apply_rope=c.arch == "llama" and not roped, partial=partial, nslabs=ns)
        if meta.is_prefill:
            qb = (meta.qb_seq, meta.qb_start) if meta.qb_seq is not None else None
            paged = None
            if meta.ctx_start is not None:  # some prompts start with cached prefix blocks
                paged = (meta.ctx_start, k_cache, v_cache, meta.block_tables)
            nd = meta.num_decode
            if nd == 0:
                return ops.flash_prefill(qkv, meta.cu_seqlens, self.hq, self.hkv, self.D, self.scale, qblocks=qb,
                                         paged=paged)
            # mixed step: decode rows through paged_decode, prefill rows through flash prefill
            o = torch.empty(qkv.shape[0], self.hq * self.D, dtype=qkv.dtype, device=qkv.device)
            ops.paged_decode(qkv[:nd], k_cache, v_cache, meta.dec_block_tables, meta.dec_seq_lens, self.hq,
                             self.hkv, self.D, self.scale, workspace=meta.decode_ws, out=o[:nd])
            op = ops.flash_prefill(qkv[nd:], meta.cu_seqlens, self.hq, self.hkv, self.D, self.scale, qblocks=qb,
                                   paged=paged, out=o[nd:])
            if op.data_ptr() != o[nd:].data_ptr():  # CPU reference paths return a fresh tensor
                o[nd:] = op
        else:
            out = ops.packed_empty(T, self.hq * self.D, self.dtype, self.device) if slabs is not None else None
            o = ops.paged_decode(qkv, k_cache, v_cache, meta.block_tables, meta.seq_lens, self.hq, self.hkv,
                                 self.D, self.scale, workspace=meta.decode_ws, out=out)
        return o

    def _mlp(self, L: dict, x: torch.Tensor, meta: AttnMeta) -> torch.Tensor:
        c = self.cfg
        if c.arch == "gpt2":
            h = ops.gelu_tanh(F.linear(x, L["w1"], L["b1"]))
            y = F.linear(h, L["w2"])
            if self.rank == 0:
                y += L["b2"]
            return tp_all_reduce(y, self.ps)
        if c.is_moe:
            if meta.is_prefill and self.tp > 1 and self.moe_comm == "a2a":
                return self._moe_a2a(L, x)
            if not meta.is_prefill and self.tp > 1 and self.moe_decode == "a2a":
                return self._moe_a2a_decode(L, x)
            return tp_all_reduce(self._moe(L, x, meta), self.ps)
        if self._w13_il:
            h = ops.prefill_linear(x, L["w13"], swiglu=self._swg)
        else:
            h = ops.silu_mul(F.linear(x, L["w13"]), interleaved=False)
        return tp_all_reduce(ops.prefill_linear(h, L["w2"]), self.ps)

    def _moe(self, L: dict, x: torch.Tensor, meta: AttnMeta) -> torch.Tensor:
        """Top-k MoE over this rank's experts [e_lo, e_hi).  Tokens are sorted by expert (moe_align)
        and every local expert runs on its contiguous rows in ONE grouped launch per projection
        (gemm_tile.hip / moe_gemm.hip, device-side offsets: no host sync, so a decode step beyond
        the skinny kernels' row limit stays graph-capturable).  The CPU decode form is the
        dense-masked reference (every local expert on every token, scaled by its routing weight)."""
        c = self.cfg
        T = x.shape[0]
        K = c.top_k_experts
        ids, w, _ = ops.moe_router(x, L["router"], K, True)
        if not meta.is_prefill and not (self._moe_grouped and x.is_cuda):
            # CPU reference of the decode form (the GPU takes the routed grouped path below, which
            # needs no host sync either and runs only the (token, expert) pairs that were chosen)
            wd = torch.zeros(T, c.n_experts, dtype=torch.float32, device=x.device)
            wd.scatter_(1, ids.long(), w)
            out = torch.zeros(T, c.d_model, dtype=torch.float32, device=x.device)
            for j, e in enumerate(range(self.e_lo, self.e_hi)):
                h = ops.silu_mul(F.linear(x, self._expert(L, "w13", j)), interleaved=self._w13_il)
                out += F.linear(h, self._expert(L, "w2", j)).float() * wd[:, e:e + 1]
            return out.to(x.dtype)
        offsets, sorted_idx, inv_idx = ops.moe_align(ids, c.n_experts)
        xs = ops.gather_rows(x, sorted_idx, K)
        if self._moe_grouped and x.is_cuda:
            # every local expert in ONE grouped launch per projection, driven by the device-side
            # offsets (ops/csrc/moe_gemm.hip): no host sync, no per-expert loop
            offl = offsets[self.e_lo:self.e_hi + 1]
            part = self.tp > 1  # other ranks' experts' rows stay zero
            if self._w13_il:
                h = ops.moe_grouped_gemm(xs, L["w13"], offl, swiglu=self._swg, zero_fill=part)
            else:
                h = ops.silu_mul(ops.moe_grouped_gemm(xs, L["w13"], offl, zero_fill=part))
            ys = ops.moe_grouped_gemm(h, L["w2"], offl, zero_fill=part)
            return ops.moe_combine(ys, inv_idx, w, T)
        ys = torch.zeros_like(xs)
        off = offsets.tolist()  # one host sync per MoE layer (the per-expert hipBLASLt loop)
        for j, e in enumerate(range(self.e_lo, self.e_hi)):
            a, b = off[e], off[e + 1]
            if b > a:
                h = ops.silu_mul(F.linear(xs[a:b], self._expert(L, "w13", j)), interleaved=self._w13_il)
                ys[a:b] = F.linear(h, self._expert(L, "w2", j))
        return ops.moe_combine(ys, inv_idx, w, T)

    def _moe_a2a(self, L: dict, x: torch.Tensor) -> torch.Tensor:
        """Expert-parallel MoE with all-to-all dispatch / combine, for prefill
        at TP>1.  Activations arrive replicated (tensor-parallel attention); rank r routes its
        1/tp slice of the tokens, sends every (token, expert) row to the rank owning the expert,
        the owners sort what they received by local expert and run all local experts in one grouped
        GEMM launch per projection (host sync only for the all-to-all sizes), the results travel back by the reverse all-to-all, are combined with the
        routing weights, and the slices are all-gathered to the replicated layout the next layer's
        attention expects.  Decode keeps the graph-capturable replicated form (_moe + all-reduce):
        all-to-all splits are data-dependent and need a host sync."""
        c = self.cfg
        T, K, P, r = x.shape[0], c.top_k_experts, self.tp, self.rank
        epr = c.n_experts // P
        chunk = -(-T // P)
        t0, t1 = min(T, r * chunk), min(T, (r + 1) * chunk)
        n = t1 - t0
        xs = x[t0:t1]
        ids, w, _ = ops.moe_router(xs, L["router"], K, True)
        offsets, sorted_idx, inv_idx = ops.moe_align(ids, c.n_experts)
        send = ops.gather_rows(xs, sorted_idx, K) if n else xs.new_zeros(0, c.d_model)
        send_exp = ids.reshape(-1)[sorted_idx.long()].to(torch.int64)
        off = offsets.tolist()  # host sync: all-to-all split sizes
        send_counts = [off[(p + 1) * epr] - off[p * epr] for p in range(P)]
        cnt = torch.tensor(send_counts, dtype=torch.int64, device=x.device)
        rcnt = torch.empty_like(cnt)
        tp_all_to_all(rcnt, cnt, [1] * P, [1] * P, self.ps)
        recv_counts = rcnt.tolist()
        nrecv = sum(recv_counts)
        recv = x.new_empty(nrecv, c.d_model)
        tp_all_to_all(recv, send, recv_counts, send_counts, self.ps)
        recv_exp = torch.empty(nrecv, dtype=torch.int64, device=x.device)
        tp_all_to_all(recv_exp, send_exp, recv_counts, send_counts, self.ps)
        # the received rows arrive grouped by source rank; order them by local expert and run all
        # local experts in one grouped launch per projection (device offsets, no further sync)
        order = torch.argsort(recv_exp, stable=True)
        counts = torch.bincount(recv_exp[order] - self.e_lo, minlength=epr)
        loc_off = torch.zeros(epr + 1, dtype=torch.int32, device=x.device)
        loc_off[1:] = torch.cumsum(counts, 0).to(torch.int32)
        xs_l = recv[order]
        if self._w13_il:
            h = ops.moe_grouped_gemm(xs_l, L["w13"], loc_off, swiglu=self._swg, zero_fill=False)
        else:
            h = ops.silu_mul(ops.moe_grouped_gemm(xs_l, L["w13"], loc_off, zero_fill=False))
        y = torch.empty_like(recv)
        y[order] = ops.moe_grouped_gemm(h, L["w2"], loc_off, zero_fill=False)
        back = x.new_empty(n * K, c.d_model)
        tp_all_to_all(back, y, send_counts, recv_counts, self.ps)
        out = ops.moe_combine(back, inv_idx, w, n) if n else back[:0]
        if n < chunk:  # equal-size blocks for the all-gather
            out = torch.cat([out, out.new_zeros(chunk - n, c.d_model)])
        return tp_all_gather_rows(out, self.ps)[:T]

    def _a2a_equal(self, x: torch.Tensor) -> torch.Tensor:
        """All-to-all of equal blocks x [P, ...] -> out[p] = rank p's x[this rank]: the IPC kernel
        (custom_ar.hip, one launch, graph-capturable) on the GPU, else the group backend."""
        car = self.ps.custom_ar
        if car is not None and x.is_cuda and car.fits_a2a(x):
            return car.all_to_all(x)
        out = torch.empty_like(x)
        n = x.shape[0]
        tp_all_to_all(out.view(n, -1), x.reshape(n, -1), [1] * n, [1] * n, self.ps)
        return out

    def _moe_a2a_decode(self, L: dict, x: torch.Tensor) -> torch.Tensor:
        """Expert-parallel MoE for DECODE steps with static shapes, so the
        step stays capturable in a hipGraph: rank r routes its ceil(M/P) slice of the (replicated)
        rows; every (token, slot) pair goes to the rank owning its expert through a fixed-capacity
        all-to-all (cap = slice x top-k rows per rank pair, zero rows where a pair goes elsewhere;
        the IPC all-to-all kernel on the GPU, custom_ar.hip); the owner runs its local experts on
        what it received on the grouped skinny MFMA kernels (one launch for gate/up + SwiGLU of
        every local expert, one for their down projections into split-K slabs weighted one-hot by
        each row's expert - the slab sum IS the per-row expert selection), in chunks of up to 128
        rows (the row-major grouped kernel's 8-m-tile form: one weight stream per step at batch 64);
        the results return by the reverse all-to-all, are weighted and summed per token, and the
        slices are all-gathered.  Against the replicated form (every rank runs its experts on
        every token, then one all-reduce) it computes only routed pairs, streams the local expert
        weights once per 128-row chunk of the P x cap x K received rows (once per step at batch 64,
        TP 2), and moves two all-to-alls plus an all-gather; the replicated form stays the default
        (K8SLLM_MOE_DECODE=a2a selects this one)."""
        c = self.cfg
        P, r, K, d = self.tp, self.rank, c.top_k_experts, c.d_model
        epr = c.n_experts // P
        M = x.shape[0]
        cap = -(-M // P)
        if M < P * cap:
            x = torch.cat([x, x.new_zeros(P * cap - M, d)])
        xs = x[r * cap:(r + 1) * cap]
        ids, w, _ = ops.moe_router(xs, L["router"], K, True)  # [cap, K]
        ids = ids.long()
        npair = cap * K
        pair_x = xs.repeat_interleave(K, dim=0)  # [cap*K, d], pair j = (token j // K, slot j % K)
        dest = (ids // epr).view(-1)  # [cap*K]
        sel = dest.unsqueeze(0) == torch.arange(P, device=x.device).unsqueeze(1)  # [P, cap*K]
        send = pair_x.unsqueeze(0) * sel.unsqueeze(-1).to(x.dtype)
        # expert ids travel as bf16 (exact small integers, -1 = no pair), padded to 8 per block
        ne = -(-npair // 8) * 8
        send_e = torch.full((P, ne), -1.0, dtype=x.dtype, device=x.device)
        send_e[:, :npair] = torch.where(sel, (ids.view(-1) % epr).unsqueeze(0), torch.full_like(sel, -1,
                                                                                              dtype=torch.long)).to(x.dtype)
        recv = self._a2a_equal(send.contiguous())
        recv_e = self._a2a_equal(send_e)
        R = P * npair
        rows = recv.view(R, d)
        re = recv_e[:, :npair].reshape(-1).float()
        onehot = (re.unsqueeze(1) == torch.arange(epr, device=x.device, dtype=torch.float32).unsqueeze(0)).float()
        ws = self._skinny_ws
        if ws is not None and "w13_pg" not in L and "w13_dg" in L:
            # ONE_LAYOUT: the shared-A grouped decode GEMM over the packed experts, 64 rows a launch
            y = torch.empty(R, d, dtype=x.dtype, device=x.device)
            E = L["w13_dg"].shape[0]
            for c0 in range(0, R, ops.SKINNY_MAX_M):
                mc = min(ops.SKINNY_MAX_M, R - c0)
                act = torch.empty((E, -(-mc // 16), L["w13_dg"].shape[1] // 4, 64, 8), dtype=x.dtype, device=x.device)
                ops.dec_gemm_grouped(ops.pack_activation(rows[c0:c0 + mc]), L["w13_dg"], 2, mc, out=act)
                ns = ops.dec_gemm_grouped(act, L["w2_dg"], 0, mc, workspace=ws, row_w=onehot[c0:c0 + mc].contiguous())
                ops.reduce_slabs(ws, ns, mc, d, dtype=x.dtype, out=y[c0:c0 + mc])
        elif ws is not None and "w13_pg" in L:
            y = torch.empty(R, d, dtype=x.dtype, device=x.device)
            # up to 128 rows per grouped launch over the row-major expert weights: at decode batch
            # 64 and TP=2 the P x cap x top-k = 128 received rows stream each local expert ONCE
            step = (ops.SKINNY_GROUPED_MAX_M if L["w13_pg"].dim() == 3 and epr > 1 and x.is_cuda
                    else ops.SKINNY_MAX_M)
            for c0 in range(0, R, step):
                mc = min(step, R - c0)
                act = ops.skinny_grouped_swiglu(ops.pack_activation(rows[c0:c0 + mc]), L["w13_pg"], rows=mc)
                ns = ops.skinny_grouped_slabs(act, L["w2_pg"], ws, mc, onehot[c0:c0 + mc].contiguous(), splits=1)
                ops.reduce_slabs(ws, ns, mc, d, dtype=x.dtype, out=y[c0:c0 + mc])
        else:
            yf = torch.zeros(R, d, dtype=torch.float32, device=x.device)
            for j in range(epr):
                h = ops.silu_mul(F.linear(rows, self._expert(L, "w13", j)), interleaved=self._w13_il)
                yf += F.linear(h, self._expert(L, "w2", j)).float() * onehot[:, j:j + 1]
            y = yf.to(x.dtype)
        back = self._a2a_equal(y.view(P, npair, d))
        res = back[dest, torch.arange(npair, device=x.device)]  # [cap*K, d]
        z = (res.view(cap, K, d).float() * w.unsqueeze(-1)).sum(1).to(x.dtype)
        return tp_all_gather_rows(z, self.ps)[:M]

    def _norm(self, x: torch.Tensor, w) -> torch.Tensor:
        if isinstance(w, tuple):
            return ops.layer_norm(x, w[0], w[1], self.cfg.norm_eps)
        return ops.rms_norm(x, w, self.cfg.norm_eps)

    def forward(self, ids: torch.Tensor, meta: AttnMeta, kv_caches: Optional[list] = None) -> torch.Tensor:
        """Returns logits [rows, vocab_size] for the rows selected by ``meta.logits_idx`` (all rows
        when None)."""
        c = self.cfg
        if meta.dec_src is not None:
            if (self.tp == 1 and ids.is_cuda and c.arch != "gpt2" and self._use_skinny(meta, ids)
                    and c.d_model % 512 == 0):
                # decode front end in one launch: ids -> embedding -> layer 0's deferred-norm operands
                residual, xw, ss = ops.embed_norm_partial(ids, self.embed, self.layers[0]["attn_norm"],
                                                          meta.dec_src, meta.dec_prev)
                return self._decode_layers_skinny(None, residual, meta, kv_caches, first=(xw, (ss, c.norm_eps)))
            ids = ops.resolve_ids(ids, meta.dec_src, meta.dec_prev)
        h = self.embed_tokens(ids)
        if c.arch == "gpt2":
            h = h + self.pos_embed[meta.positions.long()]
            residual = h
            for i, L in enumerate(self.layers):
                kv = kv_caches[i] if kv_caches is not None else None
                residual = residual + self._attention(L, self._norm(residual, L["ln1"]), meta, kv)
                residual = residual + self._mlp(L, self._norm(residual, L["ln2"]), meta)
            x = residual
            if meta.logits_idx is not None:
                x = x[meta.logits_idx]
            x = self._norm(x, self.final_norm)
        else:
            residual = h
            if self._use_skinny(meta, h):
                return self._decode_layers_skinny(None, residual, meta, kv_caches)
            if self._fused_norm_ok(h):
                return self._logits(self._prefill_fused_norm(residual, meta, kv_caches))
            if meta.micro is not None and self.overlap_ok():
                return self._logits(self._prefill_overlap(residual, meta, kv_caches))
            x = ops.rms_norm(h, self.layers[0]["attn_norm"], c.norm_eps)
            n = len(self.layers)
            for i, L in enumerate(self.layers):
                kv = kv_caches[i] if kv_caches is not None else None
                y = self._attention(L, x, meta, kv)
                x = ops.fused_add_rms_norm(y, residual, L["mlp_norm"], c.norm_eps)
                y = self._mlp(L, x, meta)
                if i + 1 < n:
                    x = ops.fused_add_rms_norm(y, residual, self.layers[i + 1]["attn_norm"], c.norm_eps)
                else:
                    if meta.logits_idx is not None:
                        y = y[meta.logits_idx]
                        residual = residual[meta.logits_idx].contiguous()
                    x = ops.fused_add_rms_norm(y.contiguous(), residual, self.final_norm, c.norm_eps)
        return self._logits(x)

    def overlap_ok(self) -> bool:
        """TP > 1 dense Llama prefill may run as two overlapped micro-batches (_prefill_overlap;
        K8SLLM_TP_OVERLAP=0 disables)."""
        return (self.tp > 1 and self.cfg.arch == "llama" and not self.cfg.is_moe and bool(self.layers)
                and "bqkv" not in self.layers[0] and os.environ.get("K8SLLM_TP_OVERLAP", "1") != "0")

    def _mlp_local(self, L: dict, x: torch.Tensor) -> torch.Tensor:
        """Dense SwiGLU MLP of this rank's F shard, before the row-parallel all-reduce."""
        if self._w13_il:
            h = ops.prefill_linear(x, L["w13"], swiglu=self._swg)
        else:
            h = ops.silu_mul(F.linear(x, L["w13"]), interleaved=False)
        return ops.prefill_linear(h, L["w2"])

    def _prefill_overlap(self, residual: torch.Tensor, meta: AttnMeta, kv_caches: Optional[list]) -> torch.Tensor:
        """Tensor-parallel prefill with the row-parallel all-reduces hidden behind compute
        (SURVEY.md §2.12 C-1 / C-2): the step's sequences form two micro-batches A and B (the
        runner's split, meta.micro) and every all-reduce is issued asynchronously (RCCL runs it on
        its own stream; the consumer waits on it just before use), so per layer

            attn A, o A, [AR A] | attn B, o B, [AR B] | norm A, mlp A, [AR2 A] | norm B, mlp B, [AR2 B]

        each all-reduce runs beside the other micro-batch's next compute segment (AR2 B beside the
        next layer's attention of A).  Row-wise the arithmetic is the serial form's: the same
        GEMMs, norms and sums per row, split by sequence (attention never crosses sequences)."""
        c = self.cfg
        eps = c.norm_eps
        mA, mB, TA = meta.micro
        metas = (mA, mB)
        rs = (residual[:TA], residual[TA:])
        x0 = ops.rms_norm(residual, self.layers[0]["attn_norm"], eps)
        xs = [x0[:TA], x0[TA:]]
        pend = [None, None]  # (y, work): a micro-batch's MLP output and its all-reduce in flight
        for i, L in enumerate(self.layers):
            kv = kv_caches[i] if kv_caches is not None else None
            ys, works = [None, None], [None, None]
            for b in (0, 1):
                if pend[b] is not None:
                    y2, w2 = pend[b]
                    w2.wait()
                    xs[b] = ops.fused_add_rms_norm(y2, rs[b], L["attn_norm"], eps)
                o = self._attn_core(L, xs[b], metas[b], kv)
                ys[b] = ops.prefill_linear(o, L["wo"])
                works[b] = tp_all_reduce_async(ys[b], self.ps)
            for b in (0, 1):
                works[b].wait()
                xb = ops.fused_add_rms_norm(ys[b], rs[b], L["mlp_norm"], eps)
                y2 = self._mlp_local(L, xb)
                pend[b] = (y2, tp_all_reduce_async(y2, self.ps))
        outs = []
        for b in (0, 1):
            y2, w2 = pend[b]
            w2.wait()
            idx = metas[b].logits_idx
            outs.append(ops.fused_add_rms_norm(y2[idx].contiguous(), rs[b][idx].contiguous(), self.final_norm, eps))
        return torch.cat(outs)

    def _fused_norm_ok(self, h: torch.Tensor) -> bool:
        """Dense Llama-family prefill at TP=1 on the tile GEMMs: the RMSNorms between projections
        can live in the GEMM epilogues (``_prefill_fused_norm``)."""
        c = self.cfg
        if not h.is_cuda or c.arch != "llama" or c.is_moe or self.tp != 1 or not self._w13_il:
            return False
        if self.D != 128 or self.cos_sin is None or any(k in self.layers[0] for k in ("bqkv", "bo")):
            return False
        L = self.layers[0]
        return ops.fused_norm_ok(h.shape[0], c.d_model, ops.w_out(L["wqkv"]), ops.w_in(L["wo"]), ops.w_out(L["w13"]),
                                 ops.w_in(L["w2"]))

    def _prefill_fused_norm(self, residual: torch.Tensor, meta: AttnMeta, kv_caches: Optional[list]) -> torch.Tensor:
        """The prefill layers with every RMSNorm but the first and the final one folded into the
        tile GEMMs: the o / down epilogues add their product to the residual stream in place and
        emit (residual * next norm weight, per-128-column sums of squares); qkv (+ RoPE) and
        gate_up (+ SwiGLU) scale their rows by the resulting 1/rms - no separate fused-add RMSNorm
        pass over the [tokens, d_model] activations between projections."""
        c = self.cfg
        eps = c.norm_eps
        n = len(self.layers)
        x = ops.rms_norm(residual, self.layers[0]["attn_norm"], eps)
        ss = None
        for i, L in enumerate(self.layers):
            kv = kv_caches[i] if kv_caches is not None else None
            o = self._attn_core(L, x, meta, kv, rowscale=(ss, eps) if ss is not None else None)
            x, ss = ops.gemm_tile_resid(o, L["wo"], residual, L["mlp_norm"])
            act = ops.prefill_linear(x, L["w13"], swiglu=self._swg, rowscale=(ss, eps))
            if i + 1 < n:
                x, ss = ops.gemm_tile_resid(act, L["w2"], residual, self.layers[i + 1]["attn_norm"])
            else:
                y = ops.prefill_linear(act, L["w2"])
                if meta.logits_idx is not None:
                    y = y[meta.logits_idx]
                    residual = residual[meta.logits_idx].contiguous()
                x = ops.fused_add_rms_norm(y.contiguous(), residual, self.final_norm, eps)
        return x

    def _logits(self, x: torch.Tensor, rows: Optional[int] = None) -> torch.Tensor:
        """LM head (+ the TP all-gather of the vocab shards).  ``x``: the final-normed rows,
        row-major, or fragment-packed with ``rows`` valid rows (decode).  With a decode copy of the
        head (``lm_head_d``) up to 64 rows at a time go through gemm_decode.hip - the decode step's
        and a prefill step's last-token logits alike; hipBLASLt otherwise."""
        hd = self.lm_head_d
        if x.dim() == 4:  # packed (decode): the decode copy exists by construction
            logits = torch.empty(rows, hd.shape[0] * 16, dtype=self.dtype, device=self.device)
            ops.dec_gemm(x, hd, 1, rows, out=logits)
        elif hd is not None and x.is_cuda and x.shape[0] <= ops.SKINNY_MAX_M:
            logits = torch.empty(x.shape[0], hd.shape[0] * 16, dtype=self.dtype, device=self.device)
            ops.dec_gemm(ops.pack_activation(x), hd, 1, x.shape[0], out=logits)
        elif self.lm_head.dim() == 4:  # ONE_LAYOUT: the packed head is the only copy - 64-row chunks
            M, mc = x.shape[0], ops.SKINNY_MAX_M
            logits = torch.empty(M, hd.shape[0] * 16, dtype=self.dtype, device=self.device)
            for i in range(0, M, mc):
                m = min(mc, M - i)
                ops.dec_gemm(ops.pack_activation(x[i:i + m]), hd, 1, m, out=logits[i:i + m])
        else:
            logits = F.linear(x, self.lm_head)
        logits = tp_all_gather_last(logits, self.ps)
        if self.vocab_padded != self.cfg.vocab_size:
            logits = logits[:, : self.cfg.vocab_size]
        return logits

    # ------------------------------------------------------------------ fused decode tail
    def _use_skinny(self, meta: AttnMeta, h: torch.Tensor) -> bool:
        """Dense Llama decode at TP=1 on the GPU with <= 64 rows runs every projection through
        gemm_skinny over fragment-packed weights (see _init_skinny)."""
        return (self._skinny_ws is not None and not meta.is_prefill and h.shape[0] <= ops.SKINNY_MAX_M
                and meta.logits_idx is None and self.SKINNY_DECODE)

    def _init_skinny(self) -> None:
        """Decode-path weights.  Dense Llama (``ONE_LAYOUT``, round 6): ``_init_dec`` packs every
        projection and the LM head into the shared-A decode GEMM's fragment-packed layout
        (gemm_decode.hip) and that packed tensor REPLACES the row-major one - prefill's tile GEMM
        reads it too (Llama-3-8B: 16.1 GB resident, Llama-3-70B at TP=1: 141 GB with every
        projection on gemm_decode).  Otherwise (MoE experts, ``ONE_LAYOUT`` off) the row-major
        tensors prefill reads serve decode through gemm_skinny_rm_kernel (ops/csrc/gemm_skinny.hip:
        whole 128-B lines by LDS-DMA; a shape it does not take keeps fragment-packed copies), and
        ``_init_dec`` adds decode-only packed copies where they fit (``_want_dec``).

        w13 is stored gate/up-interleaved per 128 rows ([64 gate | 64 up], the SwiGLU epilogue's
        pairing): called on canonical [gate; up] tensors (after _build or load_checkpoint), it
        interleaves them in place and prefill's silu_mul reads the interleaved GEMM output.

        Per layer at decode (5-7 launches): qkv skinny (split-K slabs) -> paged_decode_fused (slab
        reduce, RoPE, KV write, attention) -> o skinny (slabs) -> add_norm_partial (residual add,
        deferred mlp norm) -> gate_up skinny with the SwiGLU epilogue -> down skinny (slabs) ->
        add_norm_partial.  TP>1: each row-parallel o / down tail is ONE launch with the IPC
        all-reduce (slab sum + all-reduce + residual add + RMSNorm + packed A: _tp_tail); over
        RCCL, reduce_slabs + all-reduce + fused_add_rms_norm + pack_activation.
        On the CPU the same ops run as fp32 references with the kernels' split-K slicing, so the
        control flow (and TP over gloo) is covered by the CPU tests."""
        self._skinny_ws = None
        self.lm_head_d = None
        self._rc_o = 0
        if self.lm_head.dim() == 4:
            self.lm_head = self.canonical_head().contiguous()
        if self._packed:  # re-initialised over ONE_LAYOUT weights: back to the canonical row-major form
            for L in self.layers:
                for key in ("wqkv", "wo", "w13", "w2"):
                    L[key] = self.canonical(L, key).contiguous()
            self._packed, self._swg, self._w13_il = False, True, False
        for L in self.layers:  # (re)built below from the current weights
            for key in ("wqkv_d", "wo_d", "w13_d", "w2_d", "w13_dg", "w2_dg"):
                L.pop(key, None)
        c = self.cfg
        ff = c.ffn_dim if c.is_moe else self.f_local  # experts are sharded by count (EP), not by F
        if not getattr(self, "_w13_il", False) and c.arch == "llama" and ff % 64 == 0:
            for L in self.layers:
                w = L["w13"]
                L["w13"] = (torch.stack([ops.interleave_gate_up(e) for e in w]) if w.dim() == 3
                            else ops.interleave_gate_up(w)).contiguous()
                del w
            self._w13_il = True
        self._w13_il = getattr(self, "_w13_il", False)
        # (In-launch split-K epilogues - RoPE + KV write in the qkv GEMM, residual add + norm
        # producer in the o / down GEMMs, reduced by each tile's last-arriving workgroup - measured
        # 5-6 us per layer-op SLOWER than the slab GEMM + separate reduce kernel on the row-major
        # kernel too (profiles/r03/fused_epilogues_rowmajor.jsonl) and were removed.)
        # decode RoPE + KV write inside the attention kernel (paged_decode_fused), reading the qkv
        # GEMM's split-K slabs directly: one launch per layer fewer
        self._attn_rope = self.D == 128
        if c.arch != "llama" or not self.SKINNY_DECODE or not self._w13_il:
            self._attn_rope = False
            return
        d, nq = c.d_model, (self.hq + 2 * self.hkv) * self.D
        if d % 64 or nq % 64 or (self.hq * self.D) % 32:
            self._attn_rope = False
            return
        rowmajor = (self.hq * self.D) % 64 == 0
        self.skinny_layout = "rowmajor" if rowmajor else "packed"
        keep = (lambda w: w) if rowmajor else ops.pack_skinny
        for L in self.layers:
            L["wqkv_p"] = keep(L["wqkv"])
            L["wo_p"] = keep(L["wo"])
            if c.is_moe:  # stacked per local expert for the grouped (grid.z = expert) launches
                L["w13_pg"] = L["w13"] if rowmajor else torch.stack([keep(w) for w in L["w13"]])
                L["w2_pg"] = L["w2"] if rowmajor else torch.stack([keep(w) for w in L["w2"]])
            else:
                L["w13_p"] = keep(L["w13"])
                L["w2_p"] = keep(L["w2"])
        split = ops.SKINNY_SPLITS_FORCE  # 0: the launcher picks per call (kernel and batch dependent)
        self._split_qkv = self._split_o = self._split_d = split
        self._init_dec()

        def most(N: int, K: int) -> int:
            s_rm = split if split else max(ops.skinny_auto_splits(m, N, K) for m in (1, 33, 64))
            cfg = ops.dec_config(N, K, 0) if self.layers and any(k.endswith("_d") for k in self.layers[0]) else None
            return max(s_rm, cfg[0] if cfg else 1)

        n = max(most(nq, d) * nq, most(d, self.hq * self.D) * d,
                (self.e_hi - self.e_lo) * ops.skinny_nslabs(ff, 1) * d if c.is_moe else most(d, ff) * d)
        # MoE: the EP all-to-all decode runs up to 128 received rows per grouped launch
        rows = ops.SKINNY_GROUPED_MAX_M if c.is_moe else ops.SKINNY_MAX_M
        self._skinny_ws = torch.empty(n * rows, dtype=torch.float32, device=self.device)
        self.set_decode_fusion()

    # decode buckets up to this many rows take the row-complete o projection by default: per decode
    # step 1.4 % faster at 1-2 rows, 0.9 % at 4-16, 0.4 % at 32 (profiles/r05/rc_rows_ab.jsonl;
    # batch-1 TPOT 3.14 vs 3.18 ms, latency_b1_rc_ab.md); at 64 rows its per-workgroup re-read of
    # the attention output cancels the gain (neutral)
    RC_O_MAX_ROWS = 32

    def set_decode_fusion(self, rc=None) -> None:
        """The row-complete o projection as the alternative to the decode step's first
        add_norm_partial launch (profiles/r05/README.md; bit-compatible with the slab path): the o
        projection without split-K slabs, residual add and the gate_up GEMM's norm operands in its
        epilogue (ops.dec_gemm_rc).  At 64 rows it is neutral (re-reading the attention output
        from L2 in every workgroup costs what the slab round trip did); at 1-32 rows it wins
        0.4-1.4 % per step, so ``rc=None`` (the default) turns it on for decode buckets of at most
        RC_O_MAX_ROWS rows (the hipGraphs are captured per bucket, so the choice is static per
        graph); True: every bucket; False: off.  Needs TP=1 and the decode weight copies.
        (Measured and removed in round 6's cleanup: the add-RMSNorm as the consuming GEMM's first
        phase behind a grid seam - neutral to slower - and the down projection row-complete -
        0.2-4.5 % slower at 4-32 rows; profiles/r05/README.md.)"""
        c = self.cfg
        ok = (self.tp == 1 and not c.is_moe and bool(self.layers) and "w13_d" in self.layers[0]
              and c.d_model % 512 == 0)
        rows = self.RC_O_MAX_ROWS if rc is None else (1 << 30 if rc is True else int(rc))
        self._rc_o = rows if ok and "wo_d" in self.layers[0] else 0

    def _decode_layers_skinny(self, x: torch.Tensor, residual: torch.Tensor, meta: AttnMeta,
                              kv_caches: Optional[list], first: Optional[tuple] = None) -> torch.Tensor:
        """Activations between the skinny GEMMs travel fragment-packed (whole-line A loads): the
        attention output (paged_decode) and the MLP activation (SwiGLU epilogue) are written in the
        A-operand layout, and every RMSNorm is deferred: add_norm_partial writes residual * w plus
        per-row partial sums of squares, and the consuming GEMM scales its outputs by 1/rms."""
        c, ws, n = self.cfg, self._skinny_ws, len(self.layers)
        eps = c.norm_eps
        M = residual.shape[0]
        # first = layer 0's (A operand, rownorm), already produced with the embedding (embed_norm_partial)
        xw, rn = first if first is not None else self._norm_tail(residual, None, 0, self.layers[0]["attn_norm"])
        for i, L in enumerate(self.layers):
            kv = kv_caches[i] if kv_caches is not None else None
            op = self._attn_core(L, xw, meta, kv, slabs=(ws, self._split_qkv), rows=M, rownorm=rn)
            rc = None
            if M <= self._rc_o and "w13_d" in L:
                # o projection row-complete: residual += o and the gate_up GEMM's normed input in
                # the same launch (no split-K slabs, no add_norm launch)
                rc = ops.dec_gemm_rc(op, L["wo_d"], M, residual, L["mlp_norm"], eps)
            if rc is not None:
                xw, rn = rc
                act = ops.packed_empty(M, self.f_local, self.dtype, self.device)
                ops.dec_gemm(xw, L["w13_d"], 2, M, out=act, rownorm=rn)
                ns = self._proj_slabs(L, "w2", act, M, self._split_d)
                if i + 1 < n:
                    xw, rn = self._norm_tail(residual, ws, ns, self.layers[i + 1]["attn_norm"], rows=M)
                continue
            ns = self._proj_slabs(L, "wo", op, M, self._split_o)
            if c.is_moe and self.tp > 1 and self.moe_decode == "a2a":
                # EP all-to-all MoE: residual += o (all-reduced), then the complete, replicated
                # MLP output comes back from _moe_a2a_decode
                xn = self._tp_tail(ws, ns, residual, L["mlp_norm"], packed=False)
                if xn is None:
                    xn = ops.fused_add_rms_norm(self._row_parallel_sum(ws, ns, M, residual), residual,
                                                L["mlp_norm"], eps)
                z = self._moe_a2a_decode(L, xn)
                nw = self.layers[i + 1]["attn_norm"] if i + 1 < n else self.final_norm
                xr = ops.fused_add_rms_norm(z, residual, nw, eps)
                if i + 1 < n:
                    xw, rn = ops.pack_activation(xr), None
                    continue
                return self._logits(xr)
            if c.is_moe:
                ns = self._moe_skinny(L, residual, ws, ns, M)
            else:
                xw, rn = self._norm_tail(residual, ws, ns, L["mlp_norm"], rows=M)
                if "w13_d" in L:
                    act = ops.packed_empty(M, self.f_local, self.dtype, self.device)
                    ops.dec_gemm(xw, L["w13_d"], 2, M, out=act, rownorm=rn)
                else:
                    act = ops.skinny_swiglu(xw, L["w13_p"], rows=M, packed_out=True, rownorm=rn)
                ns = self._proj_slabs(L, "w2", act, M, self._split_d)
            if i + 1 < n:
                xw, rn = self._norm_tail(residual, ws, ns, self.layers[i + 1]["attn_norm"], rows=M)
        # final norm feeds the LM head: fragment-packed for the decode GEMM (gemm_decode.hip), or
        # complete and row-major for hipBLASLt where no decode copy of the head exists
        packed = self.lm_head_d is not None
        x = self._tp_tail(ws, ns, residual, self.final_norm, packed=packed)
        if x is None:
            y = self._row_parallel_sum(ws, ns, M, residual)
            if y is None:
                out = (ops.packed_empty(M, residual.shape[1], residual.dtype, residual.device) if packed
                       else torch.empty_like(residual))
                x = ops.reduce_add_rms_norm(out, residual, ws, ns, self.final_norm, eps)
            else:
                x = ops.fused_add_rms_norm(y, residual, self.final_norm, eps)
                if packed:
                    x = ops.pack_activation(x)
        return self._logits(x, rows=M)

    def _moe_skinny(self, L: dict, residual: torch.Tensor, ws, ns: int, M: int) -> int:
        """MoE decode MLP on the grouped skinny kernels: residual += the o
        projection; the router reads the complete RMSNorm; ONE launch runs gate/up + SwiGLU of every
        local expert over every row (grid.z = expert; at decode batch sizes every expert is selected
        by some row, so the step streams every expert's weights either way), ONE launch runs their
        down projections into slabs scaled by the routing weights (0 where an expert was not
        chosen) - the caller's residual-add kernel summing the slabs is the expert combine.  Host
        sync free, so the step stays in the decode hipGraph."""
        c = self.cfg
        xn = self._tp_tail(ws, ns, residual, L["mlp_norm"], packed=False)
        xp = None  # the normed rows fragment-packed (the expert GEMMs' A operand)
        if xn is None:
            y = self._row_parallel_sum(ws, ns, M, residual)
            if y is None:
                # TP=1: one launch writes the router's row-major rows and the packed A operand
                xp = ops.packed_empty(M, c.d_model, self.dtype, self.device)
                xn = ops.reduce_add_rms_norm(torch.empty_like(residual), residual, ws, ns, L["mlp_norm"], c.norm_eps,
                                             packed_out=xp)
            else:
                xn = ops.fused_add_rms_norm(y, residual, L["mlp_norm"], c.norm_eps)
        _, _, wd = ops.moe_router(xn, L["router"], c.top_k_experts, True)
        if xp is None:
            xp = ops.pack_activation(xn)
        if "w13_dg" in L and M <= ops.SKINNY_MAX_M:  # shared-A decode GEMM over the packed expert copies
            E = L["w13_dg"].shape[0]
            act = torch.empty((E, -(-M // 16), L["w13_dg"].shape[1] // 4, 64, 8), dtype=self.dtype, device=self.device)
            ops.dec_gemm_grouped(xp, L["w13_dg"], 2, M, out=act)
            return ops.dec_gemm_grouped(act, L["w2_dg"], 0, M, workspace=ws,
                                        row_w=wd[:, self.e_lo:self.e_hi].contiguous())
        act = ops.skinny_grouped_swiglu(xp, L["w13_pg"], rows=M)
        return ops.skinny_grouped_slabs(act, L["w2_pg"], ws, M, wd[:, self.e_lo:self.e_hi].contiguous(), splits=1)

    def _proj_slabs(self, L: dict, key: str, x: Optional[torch.Tensor], rows: int, split: int,
                    rownorm: Optional[tuple] = None) -> int:
        """Split-K slabs of a decode projection into the shared workspace: the shared-A decode
        GEMM over the packed copy ``L[key + "_d"]`` where one exists, else gemm_skinny over
        ``L[key + "_p"]``.  Returns the slab count."""
        wd = L.get(key + "_d")
        if wd is not None:
            return ops.dec_gemm(x, wd, 0, rows, workspace=self._skinny_ws, rownorm=rownorm)
        return ops.skinny_slabs(x, L[key + "_p"], self._skinny_ws, split, rows=rows, rownorm=rownorm)

    def _want_dec(self) -> set:
        """Which decode-only fragment-packed copies gemm_decode.hip gets (``DECODE_GEMM`` = auto |
        dec | rm): a subset of {"head", "attn", "mlp", "experts"}.  auto, on the GPU, with W the
        weights' bytes: the LM head always (<= 2.1 GB, Llama-3-70B); the attention projections
        while W + their copies fit 70 % of the device; a dense MLP while 2W fits half of it
        (Llama-3-8B: 16 GB of 288); MoE experts while 2W fits 70 % (Mixtral-8x7B at TP=1: 93 + 93
        GB).  Llama-3-70B at TP=1 (141 GB) would get head + attention copies (+24 GB) and keep its
        MLP on the row-major skinny kernel - but dense Llama now runs ONE_LAYOUT: every projection
        is packed and the packed tensor is the only copy (no extra memory at any size); Mixtral's
        experts too."""
        mode = self.DECODE_GEMM
        if mode in ("rm", "0", "off") or self.cfg.arch != "llama":
            return set()
        if mode in ("dec", "1", "on") or self.device.type != "cuda" or self._one_layout_wanted():
            return {"head", "attn", "mlp", "experts"}
        total = torch.cuda.get_device_properties(self.device).total_memory
        w = self.num_local_params() * 2
        attn = sum((L["wqkv"].numel() + L["wo"].numel()) * 2 for L in self.layers)
        parts = {"head"}
        if w + attn <= 0.7 * total:
            parts.add("attn")
        if self.cfg.is_moe:
            if 2 * w <= 0.7 * total:
                parts.add("experts")
        elif 2 * w <= total // 2:
            parts.add("mlp")
        return parts

    def _one_layout_wanted(self) -> bool:
        """ONE_LAYOUT applies: a Llama-family model (dense or MoE) whose projections all have a
        decode configuration (the shapes are the same in every layer, so layer 0 decides)."""
        c = self.cfg
        if not (self.ONE_LAYOUT and c.arch == "llama" and self.layers and self.SKINNY_DECODE
                and self.DECODE_GEMM not in ("rm", "0", "off")
                and (self.device.type == "cuda" or self.ONE_LAYOUT == "force")):
            return False
        L = self.layers[0]
        if L["wqkv"].dim() != 2 or L["w13"].dim() != (3 if c.is_moe else 2):
            return False
        (nq, d), (f2, _) = L["wqkv"].shape, L["w13"].shape[-2:]
        attn = ops.dec_available(nq, d, 0) and ops.dec_available(d, nq - 2 * self.hkv * self.D, 0)
        if c.is_moe:  # every local expert on the grouped (grid.z = expert) decode GEMM and the grouped tile GEMM
            E = L["w13"].shape[0]
            mlp = (ops.dec_config(f2, d, 2, experts=E) is not None
                   and ops.dec_config(d, f2 // 2, 0, experts=E) is not None)
        else:
            mlp = ops.dec_available(f2, d, 2) and ops.dec_available(d, f2 // 2, 0)
        return attn and mlp and d % 256 == 0 and f2 % 256 == 0

    def _expert(self, L: dict, key: str, j: int) -> torch.Tensor:
        """Local expert j's weight row-major as the per-expert fallback paths read it (w13 in the
        ``_w13_il`` pairing), whatever the resident layout (ONE_LAYOUT: packed [E, N/16, K/32, 64, 8])."""
        w = L[key][j]
        if w.dim() == 2:
            return w
        w = ops.unpack_skinny(w)
        if key == "w13":
            w = ops.deinterleave_gate_up8(w)
            return ops.interleave_gate_up(w) if self._w13_il else w
        return w

    def canonical_head(self) -> torch.Tensor:
        """The LM head as row-major [vocab shard, d] (ONE_LAYOUT keeps only its packed copy)."""
        h = self.lm_head
        return ops.unpack_skinny(h) if h.dim() == 4 else h

    def canonical(self, L: dict, key: str) -> torch.Tensor:
        """A dense projection as the row-major [out, in] weight of the reference / the checkpoint
        format (w13 as [gate; up]), whatever its resident layout (row-major, gate/up interleaved
        per 128 rows, or the one fragment-packed copy)."""
        w = L[key]
        if w.dim() == 5 or (w.dim() == 3 and self.cfg.is_moe):  # MoE experts [E, ...]
            return torch.stack([self._canon2(e, key, e.dim() == 4) for e in w])
        return self._canon2(w, key, w.dim() == 4)

    def _canon2(self, w: torch.Tensor, key: str, packed: bool) -> torch.Tensor:
        if packed:  # ONE_LAYOUT: fragment-packed (w13: interleaved per 16 rows)
            w = ops.unpack_skinny(w)
            return ops.deinterleave_gate_up8(w) if key == "w13" else w
        return ops.deinterleave_gate_up(w) if key == "w13" and self._w13_il else w

    @torch.no_grad()
    def copy_weights_from(self, src: "CausalLM") -> None:
        """Copy ``src``'s weights into this model (same config and TP shard; any device / dtype /
        resident layout on either side - the dense projections go through their canonical form),
        then rebuild this model's derived decode copies.  Used to give an fp32 CPU reference the
        GPU model's exact weights."""
        dense = ("wqkv", "wo", "w13", "w2")
        self.embed.copy_(src.embed)
        if self.lm_head is not self.embed:
            h = src.canonical_head().to(self.lm_head.device)
            self.lm_head.copy_(ops.pack_skinny(h) if self.lm_head.dim() == 4 else h)
        for a, b in zip(self.final_norm if isinstance(self.final_norm, tuple) else (self.final_norm,),
                        src.final_norm if isinstance(src.final_norm, tuple) else (src.final_norm,)):
            a.copy_(b)
        derived = False
        for Ld, Ls in zip(self.layers, src.layers):
            for k, v in Ld.items():
                if k.endswith(("_p", "_pg", "_d", "_dg")):
                    derived = True
                    continue
                if k in dense and (self._packed or src._packed):
                    w = src.canonical(Ls, k).to(v.device)
                    ws = list(w) if w.dim() == 3 else [w]  # MoE: per expert
                    vs = list(v) if v.dim() in (3, 5) else [v]
                    for vd, wd in zip(vs, ws):
                        if vd.dim() == 4:
                            vd.copy_(ops.pack_skinny(ops.interleave_gate_up8(wd) if k == "w13" else wd))
                        else:
                            vd.copy_(ops.interleave_gate_up(wd) if k == "w13" and self._w13_il else wd)
                elif isinstance(v, tuple):
                    for a, b in zip(v, Ls[k]):
                        a.copy_(b)
                else:
                    v.copy_(Ls[k])
        if derived and not self._packed:  # separate decode copies (two-layout / MoE) are stale now
            self._init_skinny()

    def _init_dec(self) -> None:
        """Packed copies for the shared-A decode GEMM, per projection where gemm_decode has a
        launch configuration for its shape (ops.dec_config): wqkv_d / wo_d / w2_d
        ([N/16, K/32, 64, 8]), w13_d (gate/up interleaved per 16 rows as [8 gate | 8 up]), and the
        LM head; MoE expert stacks w13_dg / w2_dg ([E, ...], grid.z = expert).  ONE_LAYOUT (Llama
        and Mixtral): the packed copy REPLACES the row-major tensor layer by layer (peak memory =
        the weights + one layer's copy) and prefill reads it too; otherwise prefill keeps reading
        the row-major tensors."""
        self.lm_head_d = None
        parts = self._want_dec()
        c = self.cfg
        one = self._one_layout_wanted()
        for L in self.layers:
            keys = (("wqkv", "wo") if "attn" in parts else ()) + (("w2",) if "mlp" in parts and not c.is_moe else ())
            for key in keys:
                N, K = L[key].shape
                if ops.dec_available(N, K, 0):
                    L[key + "_d"] = ops.pack_skinny(L[key])
            if "mlp" in parts and not c.is_moe:
                w = ops.deinterleave_gate_up(L["w13"]) if self._w13_il else L["w13"]
                if ops.dec_available(w.shape[0], w.shape[1], 2):
                    L["w13_d"] = ops.pack_skinny(ops.interleave_gate_up8(w))
                del w
            if one and not c.is_moe:
                for key in ("wqkv", "wo", "w13", "w2"):
                    L[key] = L[key + "_d"]
                    L.pop(key + "_p", None)  # the skinny kernel's reference to the row-major tensor
            elif "experts" in parts and c.is_moe:  # [E, ...] stacks for the grouped (grid.z = expert) launches
                E, F2, d = L["w13"].shape
                if (ops.dec_config(F2, d, 2, experts=E) is not None
                        and ops.dec_config(d, F2 // 2, 0, experts=E) is not None):
                    L["w13_dg"] = torch.stack([ops.pack_skinny(ops.interleave_gate_up8(
                        ops.deinterleave_gate_up(w) if self._w13_il else w)) for w in L["w13"]])
                    L["w2_dg"] = torch.stack([ops.pack_skinny(w) for w in L["w2"]])
                if one:  # ONE_LAYOUT: the packed attention projections and experts are the only copies
                    for key in ("wqkv", "wo"):
                        L[key] = L[key + "_d"]
                        L.pop(key + "_p", None)
                    L["w13"], L["w2"] = L["w13_dg"], L["w2_dg"]
                    L.pop("w13_pg", None)
                    L.pop("w2_pg", None)
        N, K = ops.w_out(self.lm_head), ops.w_in(self.lm_head)
        if "head" in parts and N % 16 == 0 and K % 32 == 0 and ops.dec_available(N, K, 1):
            self.lm_head_d = self.lm_head if self.lm_head.dim() == 4 else ops.pack_skinny(self.lm_head)
            if one and self.lm_head is not self.embed:
                self.lm_head = self.lm_head_d  # ONE_LAYOUT: the packed head is the only copy too
        self._packed = one
        self._swg = 8 if one else True  # the prefill SwiGLU's gate/up interleave (gemm_tile swiglu)

    def _tp_tail(self, ws, ns: int, residual: torch.Tensor, norm_w, packed: bool) -> Optional[torch.Tensor]:
        """TP>1 on the GPU with the IPC all-reduce: the row-parallel tail (slab sum, all-reduce,
        residual add, RMSNorm, the next GEMM's input layout) as ONE fused launch
        (custom_ar.hip car_fused_tail_kernel); None where it does not apply."""
        car = self.ps.custom_ar
        M, d = residual.shape
        if self.tp == 1 or ns == 0 or car is None or not residual.is_cuda or not car.fits_tail(M, d):
            return None
        out = (ops.packed_empty(M, d, residual.dtype, residual.device) if packed
               else torch.empty_like(residual))
        return car.fused_tail(ws, ns, residual, norm_w, self.cfg.norm_eps, out, packed)

    def _row_parallel_sum(self, ws, ns: int, M: int, residual: torch.Tensor) -> Optional[torch.Tensor]:
        """TP>1: the row-parallel projection's slabs summed to bf16 and all-reduced; None at TP=1."""
        if self.tp == 1 or ns == 0:
            return None
        y = ops.reduce_slabs(ws, ns, M, residual.shape[1], dtype=residual.dtype)
        return tp_all_reduce(y, self.ps)

    def _norm_tail(self, residual: torch.Tensor, ws, ns: int, norm_w, rows: Optional[int] = None) -> tuple:
        """residual += the projection's slabs; returns (A operand for the next skinny GEMM, rownorm)."""
        eps = self.cfg.norm_eps
        xp = self._tp_tail(ws, ns, residual, norm_w, packed=True)
        if xp is not None:
            return xp, None
        y = self._row_parallel_sum(ws, ns, residual.shape[0], residual)
        if y is not None:  # TP>1: all-reduced partial sums, complete norm, packed A
            return ops.pack_activation(ops.fused_add_rms_norm(y, residual, norm_w, eps)), None
        if residual.shape[1] % 512 == 0:
            xw, ss = ops.add_norm_partial(residual, ws, ns, norm_w)
            return xw, (ss, eps)
        out = ops.packed_empty(residual.shape[0], residual.shape[1], residual.dtype, residual.device)
        return ops.reduce_add_rms_norm(out, residual, ws, ns, norm_w, eps), None


_DUMMY_CS: dict = {}


def _dummy_cs(m: CausalLM) -> torch.Tensor:
    k = (m.device, m.D)
    if k not in _DUMMY_CS:
        _DUMMY_CS[k] = torch.zeros(1, m.D, dtype=torch.float32, device=m.device)
    return _DUMMY_CS[k]
