"""Continuous-batching scheduler.

Each engine step is either a *prefill* step (admit waiting requests while the token budget and
the free KV blocks last; a prompt larger than the remaining budget is prefilled in chunks over
several steps) or a *decode* step (one token for every fully prefilled running sequence).
Prefill has priority so newly arrived diagnostic queries join the running batch at the next
step; decode steps are captured hipGraphs, so keeping them homogeneous keeps them replayable.
When the cache runs out during decode the most recently admitted sequence is preempted
(blocks freed, re-queued at the front, recomputed later) - a full cache degrades throughput, it
never fails requests ("OOM on KV-cache allocation leads to request rejection with
503, not a crash"; here it does not even reject).
"""
from __future__ import annotations

from collections import deque
from dataclasses import dataclass, field
from typing import Optional

from .block_manager import BlockManager
from .sequence import Sequence, SeqStatus


@dataclass
class SchedulerConfig:
    max_num_seqs: int = 64
    max_prefill_tokens: int = 16384
    max_model_len: int = 8192
    # chunked prefill: a prompt that does not fit the step's remaining token budget is prefilled
    # in chunks over several steps (later chunks attend the earlier ones through the paged flash
    # prefill), so every prefill step computes at most max_prefill_tokens tokens - a bound on the
    # step's activation memory and on how long running decodes wait behind a long prompt
    chunked_prefill: bool = True


@dataclass
class StepPlan:
    is_prefill: bool
    seqs: list[Sequence] = field(default_factory=list)
    preempted: list[Sequence] = field(default_factory=list)

    @property
    def empty(self) -> bool:
        return not self.seqs


class Scheduler:
    def __init__(self, cfg: SchedulerConfig, blocks: BlockManager):
        self.cfg = cfg
        self.blocks = blocks
        self.waiting: deque[Sequence] = deque()
        self.running: list[Sequence] = []

    def add(self, seq: Sequence) -> None:
        if len(seq.prompt_ids) == 0:
            raise ValueError("empty prompt")
        if len(seq.prompt_ids) >= self.cfg.max_model_len:
            raise ValueError(f"prompt of {len(seq.prompt_ids)} tokens exceeds max_model_len {self.cfg.max_model_len}")
        if self.blocks.blocks_needed(len(seq.prompt_ids) + 1) > self.blocks.num_blocks:
            raise ValueError("prompt larger than the whole KV cache")
        seq.status = SeqStatus.WAITING
        self.waiting.append(seq)

    def abort(self, seq: Sequence) -> None:
        if seq in self.running:
            self.running.remove(seq)
        try:
            self.waiting.remove(seq)
        except ValueError:
            pass
        self.blocks.free(seq)
        seq.status = SeqStatus.ABORTED

    def has_work(self) -> bool:
        return bool(self.waiting or self.running)

    def prefill_pending(self) -> bool:
        """Would the next schedule() be a prefill step?"""
        return bool(self.waiting and len(self.running) < self.cfg.max_num_seqs) or any(
            not q.prefilled for q in self.running)

    def schedule(self) -> StepPlan:
        # 1. prefill: first the next chunks of partially prefilled sequences, then newly arrived
        #    (or preempted) requests, within the step's token budget
        partial = [q for q in self.running if not q.prefilled]
        if partial or (self.waiting and len(self.running) < self.cfg.max_num_seqs):
            plan = StepPlan(is_prefill=True)
            budget = self.cfg.max_prefill_tokens
            for seq in partial:
                if budget <= 0:
                    break
                self._take_chunk(seq, budget, plan)
                budget -= seq.chunk
            while budget > 0 and self.waiting and len(self.running) < self.cfg.max_num_seqs:  # admitted join running
                seq = self.waiting[0]
                n = seq.num_tokens - self.blocks.cached_prefix_tokens(seq)  # tokens left to compute
                if n > budget and not self.cfg.chunked_prefill and plan.seqs:
                    break
                if not self.blocks.can_allocate(seq):
                    break
                self.waiting.popleft()
                self.blocks.allocate(seq)
                seq.status = SeqStatus.RUNNING
                self.running.append(seq)
                self._take_chunk(seq, budget if self.cfg.chunked_prefill else n, plan)
                budget -= seq.chunk
            if plan.seqs:
                return plan
        # 2. decode every running sequence
        plan = StepPlan(is_prefill=False)
        i = 0
        while i < len(self.running):
            seq = self.running[i]
            if self.blocks.ensure_slot(seq):
                i += 1
                continue
            victim = self.running.pop()  # youngest
            self._preempt(victim)
            plan.preempted.append(victim)
            # retry the same index (the victim may have been this very sequence)
        plan.seqs = list(self.running)
        return plan

    def _take_chunk(self, seq: Sequence, budget: int, plan: StepPlan) -> None:
        """Schedule seq's next prefill chunk (at most ``budget`` tokens) into ``plan``."""
        seq.chunk = min(seq.num_tokens - seq.num_computed, max(1, budget))
        self.blocks.publish_computed(seq, seq.num_computed + seq.chunk)
        plan.seqs.append(seq)

    @staticmethod
    def chunk_done(seq: Sequence) -> bool:
        """Account a finished prefill step for seq; True when its whole prompt is now prefilled
        (the step's sampled token is then its first output token)."""
        seq.num_computed += seq.chunk
        seq.chunk = 0
        seq.prefilled = seq.num_computed >= seq.num_tokens
        return seq.prefilled

    def _preempt(self, seq: Sequence) -> None:
        self.blocks.free(seq)
        seq.status = SeqStatus.WAITING
        seq.n_preemptions += 1
        self.waiting.appendleft(seq)

    def finish(self, seq: Sequence, reason: str) -> None:
        seq.status = SeqStatus.FINISHED
        seq.finish_reason = reason
        if seq in self.running:
            self.running.remove(seq)
        self.blocks.free(seq)

    def stats(self) -> dict:
        d = {
            "waiting": len(self.waiting),
            "running": len(self.running),
            "kv_blocks_total": self.blocks.num_blocks,
            "kv_blocks_free": self.blocks.num_free,
            "kv_usage": round(self.blocks.usage(), 4),
        }
        d.update(self.blocks.stats())
        return d


def next_plan_or_none(s: Scheduler) -> Optional[StepPlan]:
    if not s.has_work():
        return None
    p = s.schedule()
    return None if p.empty else p
