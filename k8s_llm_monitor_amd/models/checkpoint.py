"""Real-weight checkpoints: Hugging Face ``config.json`` + ``*.safetensors`` directories.

The reference calls a remote OpenAI model and ships no weights (SURVEY.md §5 "Checkpoint /
resume": "Optional safetensors loading when weights exist"); benchmarks here run random-init
weights because the GPU box has no network.  A deployment with real weights on disk points
``llm.weights`` (EngineConfig.weights) at a Hugging Face model directory:

* :func:`config_from_hf` maps ``config.json`` (``llama`` / ``mixtral`` / ``gpt2``) onto a
  :class:`ModelConfig`;
* :func:`load_checkpoint` streams the tensors (safetensors, memory-mapped, nothing executed from
  the file) into a :class:`CausalLM`, fusing q/k/v -> ``wqkv`` and gate/up -> ``w13``, cutting this
  rank's tensor-parallel / expert-parallel shard, padding the vocabulary, then re-packing the
  decode-layout weight copies;
* :func:`save_checkpoint` writes a TP=1 model back under the same Hugging Face names (exporting a
  random-init model, round-trip tests).

Name maps (HF -> this framework):

  llama / mixtral: model.embed_tokens -> embed, lm_head -> lm_head, model.norm -> final_norm,
    layers.i.self_attn.{q,k,v}_proj -> wqkv, o_proj -> wo, input_layernorm -> attn_norm,
    post_attention_layernorm -> mlp_norm, mlp.{gate,up}_proj -> w13, mlp.down_proj -> w2,
    block_sparse_moe.gate -> router, block_sparse_moe.experts.e.{w1,w3} -> w13[e], .w2 -> w2[e]
    (or the fused-expert form mlp.gate / mlp.experts.gate_up_proj / mlp.experts.down_proj)
  gpt2: transformer.wte / wpe / ln_f, h.i.ln_1 / ln_2, attn.c_attn / c_proj, mlp.c_fc / c_proj
    (Conv1D weights are stored [in, out]: transposed on load and on save)
"""
from __future__ import annotations

import json
from pathlib import Path
from typing import Iterator, Optional, Union

import torch

from .config import ModelConfig

PathLike = Union[str, Path]


# ----------------------------------------------------------------------------- config.json

def _first(d: dict, *keys, default=None):
    for k in keys:
        if k in d and d[k] is not None:
            return d[k]
    return default


def config_from_hf(hf: Union[dict, PathLike], name: Optional[str] = None) -> ModelConfig:
    """A :class:`ModelConfig` from a Hugging Face ``config.json`` (dict, file or model directory)."""
    if not isinstance(hf, dict):
        p = Path(hf)
        if p.is_dir():
            p = p / "config.json"
        hf = json.loads(p.read_text())
        name = name or p.parent.name
    mt = hf.get("model_type", "llama")
    eos = hf.get("eos_token_id")
    eos_ids = tuple(eos) if isinstance(eos, (list, tuple)) else ((eos,) if eos is not None else (2,))
    bos = hf.get("bos_token_id")
    if mt == "gpt2":
        d = hf["n_embd"]
        return ModelConfig(name=name or "gpt2-hf", arch="gpt2", vocab_size=hf["vocab_size"], d_model=d,
                           n_layers=hf["n_layer"], n_heads=hf["n_head"], n_kv_heads=hf["n_head"],
                           head_dim=d // hf["n_head"], ffn_dim=_first(hf, "n_inner", default=4 * d) or 4 * d,
                           max_position=hf.get("n_positions", 1024), norm_eps=hf.get("layer_norm_epsilon", 1e-5),
                           tie_embeddings=True, bos_id=bos if bos is not None else 50256, eos_ids=eos_ids)
    if mt not in ("llama", "mistral", "mixtral"):
        raise ValueError(f"unsupported model_type {mt!r} (llama, mistral, mixtral, gpt2)")
    d, nh = hf["hidden_size"], hf["num_attention_heads"]
    rope = hf.get("rope_parameters") or {}  # transformers >= 5 keeps theta / scaling here
    theta = _first(hf, "rope_theta", default=rope.get("rope_theta", 10000.0))
    scaling = hf.get("rope_scaling")
    if scaling is None and rope.get("rope_type", "default") not in ("default", None):
        scaling = rope
    if scaling is not None and scaling.get("rope_type", scaling.get("type")) not in ("llama3",):
        raise ValueError(f"unsupported rope scaling {scaling!r} (llama3 frequency remap only)")
    return ModelConfig(
        name=name or f"{mt}-hf", arch="llama", vocab_size=hf["vocab_size"], d_model=d,
        n_layers=hf["num_hidden_layers"], n_heads=nh, n_kv_heads=hf.get("num_key_value_heads", nh),
        head_dim=_first(hf, "head_dim", default=d // nh), ffn_dim=hf["intermediate_size"],
        max_position=hf.get("max_position_embeddings", 8192), rope_theta=float(theta), rope_scaling=scaling,
        norm_eps=hf.get("rms_norm_eps", 1e-5), n_experts=hf.get("num_local_experts", 0) if mt == "mixtral" else 0,
        top_k_experts=hf.get("num_experts_per_tok", 2), tie_embeddings=bool(hf.get("tie_word_embeddings", False)),
        bos_id=bos if bos is not None else 1, eos_ids=eos_ids)


def config_to_hf(c: ModelConfig) -> dict:
    """The inverse of :func:`config_from_hf` (what :func:`save_checkpoint` writes)."""
    if c.arch == "gpt2":
        return {"model_type": "gpt2", "architectures": ["GPT2LMHeadModel"], "vocab_size": c.vocab_size,
                "n_embd": c.d_model, "n_layer": c.n_layers, "n_head": c.n_heads, "n_inner": c.ffn_dim,
                "n_positions": c.max_position, "layer_norm_epsilon": c.norm_eps, "bos_token_id": c.bos_id,
                "eos_token_id": c.eos_ids[0], "activation_function": "gelu_new", "tie_word_embeddings": True}
    hf = {"model_type": "mixtral" if c.is_moe else "llama",
          "architectures": ["MixtralForCausalLM" if c.is_moe else "LlamaForCausalLM"],
          "vocab_size": c.vocab_size, "hidden_size": c.d_model, "num_hidden_layers": c.n_layers,
          "num_attention_heads": c.n_heads, "num_key_value_heads": c.n_kv_heads, "head_dim": c.head_dim,
          "intermediate_size": c.ffn_dim, "max_position_embeddings": c.max_position, "rope_theta": c.rope_theta,
          "rms_norm_eps": c.norm_eps, "tie_word_embeddings": c.tie_embeddings, "bos_token_id": c.bos_id,
          "eos_token_id": list(c.eos_ids) if len(c.eos_ids) > 1 else c.eos_ids[0], "hidden_act": "silu"}
    if c.rope_scaling:
        hf["rope_scaling"] = dict(c.rope_scaling)
    if c.is_moe:
        hf["num_local_experts"] = c.n_experts
        hf["num_experts_per_tok"] = c.top_k_experts
    return hf


# ----------------------------------------------------------------------------- tensor source

class SafetensorsDir:
    """Lazy name -> tensor access over every ``*.safetensors`` file of a directory (or one file),
    memory-mapped by safetensors (no code in the file is executed)."""

    def __init__(self, path: PathLike):
        from safetensors import safe_open

        p = Path(path)
        files = sorted(p.glob("*.safetensors")) if p.is_dir() else [p]
        if not files:
            raise FileNotFoundError(f"no *.safetensors under {p}")
        self._handles = [safe_open(str(f), framework="pt", device="cpu") for f in files]
        self._where = {}
        for h in self._handles:
            for k in h.keys():
                self._where[k] = h

    def keys(self) -> list[str]:
        return list(self._where)

    def __contains__(self, k: str) -> bool:
        return k in self._where

    def get(self, k: str) -> torch.Tensor:
        if k not in self._where:
            raise KeyError(f"checkpoint has no tensor {k!r}")
        return self._where[k].get_tensor(k)

    def slice_rows(self, k: str, lo: int, hi: int) -> torch.Tensor:
        """Rows [lo, hi) of a tensor without materialising the rest (safetensors slices)."""
        return self._where[k].get_slice(k)[lo:hi]


# ----------------------------------------------------------------------------- load

def load_checkpoint(model, path: PathLike, strict: bool = True) -> list[str]:
    """Fill ``model`` (a :class:`CausalLM`, any TP rank) from a Hugging Face safetensors checkpoint.
    Returns the checkpoint tensor names that were not used (``strict`` raises on missing ones)."""
    src = path if isinstance(path, SafetensorsDir) else SafetensorsDir(path)
    used: set[str] = set()
    c, dev, dt = model.cfg, model.device, model.dtype
    D, tp, r = model.D, model.tp, model.rank
    from ..parallel.comm import kv_head_range, shard_range

    def get(k: str) -> torch.Tensor:
        used.add(k)
        return src.get(k)

    def put(t: torch.Tensor) -> torch.Tensor:
        return t.to(device=dev, dtype=dt).contiguous()

    def vocab_rows(k: str) -> torch.Tensor:
        w = get(k)
        if w.shape[0] < model.vocab_padded:
            w = torch.cat([w, w.new_zeros(model.vocab_padded - w.shape[0], w.shape[1])])
        return put(w[model.v_lo:model.v_hi])

    q_lo, q_hi = shard_range(c.n_heads * D, tp, r)
    kv_lo, kv_hi = kv_head_range(c.n_kv_heads, D, tp, r)
    f_lo, f_hi = shard_range(c.ffn_dim, tp, r)

    if c.arch == "gpt2":
        pre = "transformer." if "transformer.wte.weight" in src else ""
        model.embed = vocab_rows(pre + "wte.weight")
        model.lm_head = model.embed
        model.pos_embed = put(get(pre + "wpe.weight"))
        model.final_norm = (put(get(pre + "ln_f.weight")), put(get(pre + "ln_f.bias")))
        d = c.d_model
        for i, L in enumerate(model.layers):
            p = f"{pre}h.{i}."
            L["ln1"] = (put(get(p + "ln_1.weight")), put(get(p + "ln_1.bias")))
            L["ln2"] = (put(get(p + "ln_2.weight")), put(get(p + "ln_2.bias")))
            wqkv = get(p + "attn.c_attn.weight").t()  # Conv1D [in, out] -> [out, in]
            bqkv = get(p + "attn.c_attn.bias")
            wq, wk, wv = wqkv[:d], wqkv[d:2 * d], wqkv[2 * d:]
            bq, bk, bv = bqkv[:d], bqkv[d:2 * d], bqkv[2 * d:]
            L["wqkv"] = put(torch.cat([wq[q_lo:q_hi], wk[kv_lo:kv_hi], wv[kv_lo:kv_hi]]))
            L["bqkv"] = put(torch.cat([bq[q_lo:q_hi], bk[kv_lo:kv_hi], bv[kv_lo:kv_hi]]))
            L["wo"] = put(get(p + "attn.c_proj.weight").t()[:, q_lo:q_hi])
            L["bo"] = put(get(p + "attn.c_proj.bias"))
            L["w1"] = put(get(p + "mlp.c_fc.weight").t()[f_lo:f_hi])
            L["b1"] = put(get(p + "mlp.c_fc.bias")[f_lo:f_hi])
            L["w2"] = put(get(p + "mlp.c_proj.weight").t()[:, f_lo:f_hi])
            L["b2"] = put(get(p + "mlp.c_proj.bias"))
    else:
        # the resident layout's derived tensors (decode copies; under ONE_LAYOUT the packed weights
        # themselves) go before their replacements arrive: peak memory stays ~one copy of the model
        # (Llama-3-70B at TP = 1 would not fit two)
        model.lm_head_d = None
        for L in model.layers:
            for k in [k for k in L if k.endswith(("_p", "_d", "_pg", "_dg"))]:
                del L[k]
        model.embed = vocab_rows("model.embed_tokens.weight")
        if c.tie_embeddings or "lm_head.weight" not in src:
            model.lm_head = model.embed
        else:
            model.lm_head = vocab_rows("lm_head.weight")
        model.final_norm = put(get("model.norm.weight"))
        for i, L in enumerate(model.layers):
            p = f"model.layers.{i}."
            a = p + "self_attn."
            L["wqkv"] = put(torch.cat([src.slice_rows(a + "q_proj.weight", q_lo, q_hi),
                                       src.slice_rows(a + "k_proj.weight", kv_lo, kv_hi),
                                       src.slice_rows(a + "v_proj.weight", kv_lo, kv_hi)]))
            used.update(a + n for n in ("q_proj.weight", "k_proj.weight", "v_proj.weight"))
            L["wo"] = put(get(a + "o_proj.weight")[:, q_lo:q_hi])
            L["attn_norm"] = put(get(p + "input_layernorm.weight"))
            L["mlp_norm"] = put(get(p + "post_attention_layernorm.weight"))
            if c.is_moe:
                _load_experts(model, L, p, src, get, put, used)
            else:
                m = p + "mlp."
                L["w13"] = put(torch.cat([src.slice_rows(m + "gate_proj.weight", f_lo, f_hi),
                                          src.slice_rows(m + "up_proj.weight", f_lo, f_hi)]))
                used.update((m + "gate_proj.weight", m + "up_proj.weight"))
                L["w2"] = put(get(m + "down_proj.weight")[:, f_lo:f_hi])
    unused = sorted(set(src.keys()) - used)
    rope_buffers = [k for k in unused if k.endswith("rotary_emb.inv_freq") or k.endswith("attn.bias")
                    or k.endswith("attn.masked_bias")]
    unused = [k for k in unused if k not in rope_buffers]
    if strict and unused:
        raise ValueError(f"checkpoint tensors not consumed by {c.name}: {unused[:8]}{' ...' if len(unused) > 8 else ''}")
    model._w13_il = False  # w13 was just loaded as [gate; up]
    model._init_skinny()  # interleave w13, (re)build the decode-path views from the loaded weights
    return unused


def _load_experts(model, L: dict, p: str, src: SafetensorsDir, get, put, used: set) -> None:
    c = model.cfg
    if p + "block_sparse_moe.gate.weight" in src:  # transformers < 5: one tensor per expert
        m = p + "block_sparse_moe."
        L["router"] = put(get(m + "gate.weight"))
        w13, w2 = [], []
        for e in range(model.e_lo, model.e_hi):
            w13.append(torch.cat([get(f"{m}experts.{e}.w1.weight"), get(f"{m}experts.{e}.w3.weight")]))
            w2.append(get(f"{m}experts.{e}.w2.weight"))
        L["w13"] = put(torch.stack(w13))
        L["w2"] = put(torch.stack(w2))
    else:  # fused-expert form: experts.gate_up_proj [E, 2F, d] (gate rows, then up), down_proj [E, d, F]
        m = p + "mlp."
        L["router"] = put(get(m + "gate.weight"))
        gu = get(m + "experts.gate_up_proj")
        dn = get(m + "experts.down_proj")
        if gu.shape[1] != 2 * c.ffn_dim:  # stored [E, d, 2F]
            gu = gu.transpose(1, 2)
        if dn.shape[1] != c.d_model:  # stored [E, F, d]
            dn = dn.transpose(1, 2)
        L["w13"] = put(gu[model.e_lo:model.e_hi])
        L["w2"] = put(dn[model.e_lo:model.e_hi])


# ----------------------------------------------------------------------------- save

def hf_state_dict(model) -> Iterator[tuple[str, torch.Tensor]]:
    """(Hugging Face name, tensor) pairs of a TP=1 model, un-fused (the inverse of load)."""
    if model.tp != 1:
        raise ValueError("hf_state_dict needs the whole model (tp = 1)")
    c, D = model.cfg, model.D
    V = c.vocab_size
    if c.arch == "gpt2":
        yield "transformer.wte.weight", model.embed[:V]
        yield "transformer.wpe.weight", model.pos_embed
        yield "transformer.ln_f.weight", model.final_norm[0]
        yield "transformer.ln_f.bias", model.final_norm[1]
        for i, L in enumerate(model.layers):
            p = f"transformer.h.{i}."
            yield p + "ln_1.weight", L["ln1"][0]
            yield p + "ln_1.bias", L["ln1"][1]
            yield p + "ln_2.weight", L["ln2"][0]
            yield p + "ln_2.bias", L["ln2"][1]
            yield p + "attn.c_attn.weight", L["wqkv"].t()
            yield p + "attn.c_attn.bias", L["bqkv"]
            yield p + "attn.c_proj.weight", L["wo"].t()
            yield p + "attn.c_proj.bias", L["bo"]
            yield p + "mlp.c_fc.weight", L["w1"].t()
            yield p + "mlp.c_fc.bias", L["b1"]
            yield p + "mlp.c_proj.weight", L["w2"].t()
            yield p + "mlp.c_proj.bias", L["b2"]
        return
    nq, nk = c.n_heads * D, c.n_kv_heads * D
    yield "model.embed_tokens.weight", model.embed[:V]
    if not c.tie_embeddings:
        yield "lm_head.weight", model.canonical_head()[:V]
    yield "model.norm.weight", model.final_norm
    for i, L in enumerate(model.layers):
        p = f"model.layers.{i}."
        w = model.canonical(L, "wqkv")  # row-major whatever the resident layout (ONE_LAYOUT packs it)
        yield p + "self_attn.q_proj.weight", w[:nq]
        yield p + "self_attn.k_proj.weight", w[nq:nq + nk]
        yield p + "self_attn.v_proj.weight", w[nq + nk:]
        yield p + "self_attn.o_proj.weight", model.canonical(L, "wo")
        yield p + "input_layernorm.weight", L["attn_norm"]
        yield p + "post_attention_layernorm.weight", L["mlp_norm"]
        F = c.ffn_dim

        if c.is_moe:
            m = p + "block_sparse_moe."
            yield m + "gate.weight", L["router"]
            w13s, w2s = model.canonical(L, "w13"), model.canonical(L, "w2")  # any resident layout
            for e in range(c.n_experts):
                yield f"{m}experts.{e}.w1.weight", w13s[e][:F]
                yield f"{m}experts.{e}.w3.weight", w13s[e][F:]
                yield f"{m}experts.{e}.w2.weight", w2s[e]
        else:
            w13 = model.canonical(L, "w13")
            yield p + "mlp.gate_proj.weight", w13[:F]
            yield p + "mlp.up_proj.weight", w13[F:]
            yield p + "mlp.down_proj.weight", model.canonical(L, "w2")


def save_checkpoint(model, path: PathLike, max_shard_bytes: int = 4 << 30) -> Path:
    """Write a TP=1 model as a Hugging Face directory: config.json + model-0000i-of-0000n
    .safetensors shards (+ model.safetensors.index.json when sharded)."""
    from safetensors.torch import save_file

    out = Path(path)
    out.mkdir(parents=True, exist_ok=True)
    (out / "config.json").write_text(json.dumps(config_to_hf(model.cfg), indent=2))
    shards: list[dict] = [{}]
    size = 0
    for k, t in hf_state_dict(model):
        t = t.detach().to("cpu").contiguous().clone()
        nb = t.numel() * t.element_size()
        if shards[-1] and size + nb > max_shard_bytes:
            shards.append({})
            size = 0
        shards[-1][k] = t
        size += nb
    n = len(shards)
    index = {}
    for i, sd in enumerate(shards):
        fn = "model.safetensors" if n == 1 else f"model-{i + 1:05d}-of-{n:05d}.safetensors"
        save_file(sd, str(out / fn), metadata={"format": "pt"})
        index.update({k: fn for k in sd})
    if n > 1:
        (out / "model.safetensors.index.json").write_text(json.dumps({"metadata": {}, "weight_map": index}, indent=2))
    return out
