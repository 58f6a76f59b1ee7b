"""Request / sequence state for the continuous-batching engine."""
from __future__ import annotations

import enum
import itertools
import time
from dataclasses import dataclass, field
from typing import Optional


@dataclass
class SamplingParams:
    """Defaults follow the reference's ``llm`` block (``internal/config/config.go:141-145``):
    max_tokens 2000, temperature 0.1."""

    max_tokens: int = 2000
    temperature: float = 0.1
    top_k: int = 0
    top_p: float = 1.0
    ignore_eos: bool = False
    stop_token_ids: tuple = ()


class SeqStatus(enum.Enum):
    WAITING = "waiting"
    RUNNING = "running"
    FINISHED = "finished"
    ABORTED = "aborted"


_ids = itertools.count()


@dataclass
class Sequence:
    prompt_ids: list[int]
    params: SamplingParams
    request_id: str = ""
    seq_id: int = field(default_factory=lambda: next(_ids))
    output_ids: list[int] = field(default_factory=list)
    status: SeqStatus = SeqStatus.WAITING
    block_table: list[int] = field(default_factory=list)
    finish_reason: Optional[str] = None
    # timing (seconds, time.perf_counter clock)
    t_arrival: float = field(default_factory=time.perf_counter)
    t_first_token: Optional[float] = None
    t_finish: Optional[float] = None
    n_preemptions: int = 0
    num_cached: int = 0  # leading prompt tokens whose KV came from the prefix cache (this admission)
    # chunked prefill: tokens whose KV is in the cache (prefix cache + prefill chunks run so far),
    # the chunk the current prefill step computes, and whether the whole prompt has been prefilled
    num_computed: int = 0
    chunk: int = 0
    prefilled: bool = False
    # pipelined prefill: id of the in-flight prefill step whose sampled token will be this
    # sequence's first output token (its prompt is fully computed, the token not yet read back);
    # 0 = none.  Reset whenever the sequence's blocks are freed (preemption, abort, finish).
    pending_first: int = 0
    user: object = None  # opaque payload for the caller (future, callback, ...)
    deadline: Optional[float] = None  # time.perf_counter() by which the answer is due (engine.add_request)

    @property
    def num_tokens(self) -> int:
        return len(self.prompt_ids) + len(self.output_ids)

    @property
    def all_ids(self) -> list[int]:
        return self.prompt_ids + self.output_ids

    @property
    def last_token(self) -> int:
        return self.output_ids[-1] if self.output_ids else self.prompt_ids[-1]

    def timings(self) -> dict:
        end = self.t_finish or time.perf_counter()
        ttft = (self.t_first_token - self.t_arrival) if self.t_first_token else None
        n = len(self.output_ids)
        decode_s = (end - self.t_first_token) if self.t_first_token else 0.0
        return {
            "prompt_tokens": len(self.prompt_ids),
            "completion_tokens": n,
            "latency_ms": round((end - self.t_arrival) * 1e3, 3),
            "ttft_ms": round(ttft * 1e3, 3) if ttft is not None else None,
            "decode_tokens_per_s": round((n - 1) / decode_s, 2) if n > 1 and decode_s > 0 else None,
            "preemptions": self.n_preemptions,
        }
