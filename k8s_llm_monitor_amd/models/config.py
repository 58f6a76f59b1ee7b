"""Model architecture presets for the in-process diagnostic LLM.

The reference never runs a model: its ``llm:`` block names a remote OpenAI model
(``internal/config/config.go:141-145``, provider ``openai``, model ``gpt-4``).  BASELINE.json's
configs name the architectures this framework serves instead; their public hyper-parameters are
recorded in SURVEY.md §2.12.  Weights are random-initialised (no checkpoints on the GPU box), so a
preset is all that is needed to build a model of the right shape.
"""
from __future__ import annotations

import dataclasses
from dataclasses import dataclass, field
from typing import Optional


@dataclass(frozen=True)
class ModelConfig:
    name: str
    arch: str  # "llama" (Llama-3 / Mixtral) or "gpt2"
    vocab_size: int
    d_model: int
    n_layers: int
    n_heads: int
    n_kv_heads: int
    head_dim: int
    ffn_dim: int
    max_position: int = 8192
    rope_theta: float = 500000.0
    rope_scaling: Optional[dict] = None
    norm_eps: float = 1e-5
    n_experts: int = 0  # > 0: mixture-of-experts MLP (Mixtral)
    top_k_experts: int = 2
    tie_embeddings: bool = False
    bos_id: int = 128000
    eos_ids: tuple = (128001, 128009)
    extra: dict = field(default_factory=dict)

    @property
    def is_moe(self) -> bool:
        return self.n_experts > 0

    @property
    def q_dim(self) -> int:
        return self.n_heads * self.head_dim

    @property
    def kv_dim(self) -> int:
        return self.n_kv_heads * self.head_dim

    def num_params(self) -> int:
        d, f, L = self.d_model, self.ffn_dim, self.n_layers
        attn = d * (self.q_dim + 2 * self.kv_dim) + self.q_dim * d
        mlp = 3 * d * f * (self.n_experts if self.is_moe else 1) + (d * self.n_experts if self.is_moe else 0)
        if self.arch == "gpt2":
            mlp = 2 * d * f
        emb = self.vocab_size * d * (1 if self.tie_embeddings else 2)
        return L * (attn + mlp) + emb

    def vocab_size_padded(self, tp: int = 1) -> int:
        """Vocab rounded up to a multiple of 64*tp (vocab-parallel shards stay wave-aligned)."""
        m = 64 * tp
        return (self.vocab_size + m - 1) // m * m

    def kv_bytes_per_token(self, dtype_bytes: int = 2) -> int:
        return 2 * self.n_layers * self.kv_dim * dtype_bytes

    def replace(self, **kw) -> "ModelConfig":
        return dataclasses.replace(self, **kw)


PRESETS: dict[str, ModelConfig] = {}


def _reg(c: ModelConfig) -> ModelConfig:
    PRESETS[c.name] = c
    return c


# BASELINE.json config 1: CPU plumbing model.
GPT2_SMALL = _reg(ModelConfig(
    name="gpt2-small", arch="gpt2", vocab_size=50257, d_model=768, n_layers=12, n_heads=12, n_kv_heads=12,
    head_dim=64, ffn_dim=3072, max_position=1024, norm_eps=1e-5, tie_embeddings=True, bos_id=50256,
    eos_ids=(50256,)))

# BASELINE.json configs 2-3: the headline model.
LLAMA3_8B = _reg(ModelConfig(
    name="llama-3-8b", arch="llama", vocab_size=128256, d_model=4096, n_layers=32, n_heads=32, n_kv_heads=8,
    head_dim=128, ffn_dim=14336, max_position=8192, rope_theta=500000.0))

# BASELINE.json config 4: root-cause model, TP=8.
LLAMA3_70B = _reg(ModelConfig(
    name="llama-3-70b", arch="llama", vocab_size=128256, d_model=8192, n_layers=80, n_heads=64, n_kv_heads=8,
    head_dim=128, ffn_dim=28672, max_position=8192, rope_theta=500000.0))

# BASELINE.json config 5: anomaly-detection MoE model.
MIXTRAL_8X7B = _reg(ModelConfig(
    name="mixtral-8x7b", arch="llama", vocab_size=32000, d_model=4096, n_layers=32, n_heads=32, n_kv_heads=8,
    head_dim=128, ffn_dim=14336, max_position=32768, rope_theta=1e6, n_experts=8, top_k_experts=2,
    bos_id=1, eos_ids=(2,)))

# Small shapes with the same structure, for CPU tests and GPU smoke runs.
LLAMA_TINY = _reg(ModelConfig(
    name="llama-tiny", arch="llama", vocab_size=512, d_model=256, n_layers=2, n_heads=4, n_kv_heads=2,
    head_dim=64, ffn_dim=512, max_position=1024, rope_theta=10000.0, bos_id=1, eos_ids=(2,)))

LLAMA_TINY128 = _reg(ModelConfig(
    name="llama-tiny-d128", arch="llama", vocab_size=1024, d_model=512, n_layers=2, n_heads=8, n_kv_heads=2,
    head_dim=128, ffn_dim=1024, max_position=2048, rope_theta=500000.0, bos_id=1, eos_ids=(2,)))

MIXTRAL_TINY_D128 = _reg(ModelConfig(  # head_dim 128: the HIP attention kernels' shape, for GPU tests
    name="mixtral-tiny-d128", arch="llama", vocab_size=1024, d_model=512, n_layers=2, n_heads=8, n_kv_heads=2,
    head_dim=128, ffn_dim=1024, max_position=2048, rope_theta=1000000.0, n_experts=4, top_k_experts=2,
    bos_id=1, eos_ids=(2,)))

MIXTRAL_TINY = _reg(ModelConfig(
    name="mixtral-tiny", arch="llama", vocab_size=512, d_model=256, n_layers=2, n_heads=4, n_kv_heads=2,
    head_dim=64, ffn_dim=256, max_position=1024, rope_theta=10000.0, n_experts=4, top_k_experts=2,
    bos_id=1, eos_ids=(2,)))

MIXTRAL_TINY_E8 = _reg(ModelConfig(  # 8 query heads, 8 experts: TP / EP 8 parity tests on CPU
    name="mixtral-tiny-e8", arch="llama", vocab_size=512, d_model=256, n_layers=2, n_heads=8, n_kv_heads=2,
    head_dim=32, ffn_dim=256, max_position=1024, rope_theta=10000.0, n_experts=8, top_k_experts=2,
    bos_id=1, eos_ids=(2,)))

GPT2_TINY = _reg(ModelConfig(
    name="gpt2-tiny", arch="gpt2", vocab_size=512, d_model=128, n_layers=2, n_heads=2, n_kv_heads=2,
    head_dim=64, ffn_dim=512, max_position=512, tie_embeddings=True, bos_id=0, eos_ids=(0,)))

_ALIASES = {
    "gpt2": "gpt2-small", "gpt-2": "gpt2-small", "llama3-8b": "llama-3-8b", "meta-llama-3-8b": "llama-3-8b",
    "llama-3.1-8b": "llama-3-8b", "llama3-70b": "llama-3-70b", "mixtral": "mixtral-8x7b",
    "mixtral-8x7b-v0.1": "mixtral-8x7b",
}


def get_config(name: str) -> ModelConfig:
    key = name.strip().lower()
    key = _ALIASES.get(key, key)
    if key not in PRESETS:
        raise KeyError(f"unknown model preset {name!r}; known: {sorted(PRESETS)}")
    return PRESETS[key]
