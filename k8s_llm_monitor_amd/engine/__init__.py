"""Continuous-batching inference engine (paged KV cache, hipGraph decode, TP over RCCL)."""
from .engine import EngineConfig, EngineOverloaded, EngineService, EngineUnavailable, LLMEngine  # noqa: F401
from .sequence import SamplingParams, Sequence, SeqStatus  # noqa: F401
