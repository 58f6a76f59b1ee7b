"""Continuous-batching scheduler.

A step is one of
* *decode*  - one token for every fully prefilled running sequence (replayed from a hipGraph);
* *prefill* - prompt chunks of newly admitted (or partially prefilled) sequences within the
  step's token budget; a prompt larger than the remaining budget is prefilled in chunks;
* *mixed*   - prefill chunks AND one decode token for every running sequence, in one forward
  (SURVEY.md §7.2 step 10): the decode rows ride along the prefill GEMMs, so running answers keep
  streaming while new queries are admitted instead of stalling behind every prefill step.  The
  prefill budget of a mixed step is ``mixed_prefill_tokens`` (a bound on the TPOT hiccup a new
  arrival costs the running decodes); a prefill-only step uses ``max_prefill_tokens``.

Burst policy: while the prefill backlog is larger than one step's budget (a burst of arrivals),
steps are prefill-only - decode rows riding along would finish early but cannot shorten the burst,
and mixed steps cost more than the prefill they carry - for at most ``max_decode_stall_steps``
consecutive steps, after which one mixed step runs the decodes (so sustained overload cannot starve
them).  With a backlog of at most one step (steady arrivals) every prefill step is mixed.

When the KV cache runs out during decode the most recently admitted sequence is preempted (blocks
freed, re-queued at the front, recomputed later).  Admission of a new sequence requires its
blocks (fresh + prefix-cache hits parked in the LRU) to be free beyond a small watermark; the
serving layer (EngineService) bounds the waiting queue and rejects with 503 beyond it
("OOM on KV-cache allocation leads to request rejection with 503, not a crash").
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
    # mixed prefill+decode steps (see the module docstring); 0 = prefill steps stall decodes
    mixed_prefill_tokens: int = 16384
    # burst policy (module docstring): prefill-only steps while decodes wait, at most this many in
    # a row; 0 = always mix
    max_decode_stall_steps: int = 8


@dataclass
class StepPlan:
    """``is_prefill``: the step runs the eager prefill path over ``seqs`` (prompt chunks), plus one
    token for each of ``decode`` (a mixed step).  Otherwise ``seqs`` are the decode rows."""

    is_prefill: bool
    seqs: list[Sequence] = field(default_factory=list)
    preempted: list[Sequence] = field(default_factory=list)
    decode: list[Sequence] = field(default_factory=list)
    chunks: list[int] = field(default_factory=list)  # per-seq chunk sizes, kept for the trace

    @property
    def is_mixed(self) -> bool:
        return self.is_prefill and bool(self.decode)

    @property
    def empty(self) -> bool:
        return not self.seqs


class Scheduler:
    def __init__(self, cfg: SchedulerConfig, blocks: BlockManager):
        self.cfg = cfg
        self.blocks = blocks
        self.waiting: deque[Sequence] = deque()
        self.running: list[Sequence] = []
        self._stalled = 0  # consecutive prefill-only steps taken while decode rows were ready
        # optional admission gate ``(seq, running_after) -> bool`` (EngineService: deadline-feasible
        # admission); False keeps the head of the queue waiting (FIFO: nothing behind it starts)
        self.admit_gate = None

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
            not q.prefilled and not q.pending_first for q in self.running)

    def prefill_backlog(self) -> int:
        """Prompt tokens still to prefill: partially prefilled running sequences plus the waiting
        requests that fit the free sequence slots."""
        n = sum(q.num_tokens - q.num_computed for q in self.running if not q.prefilled and not q.pending_first)
        free = self.cfg.max_num_seqs - len(self.running)
        for i, q in enumerate(self.waiting):
            if i >= free:
                break
            n += q.num_tokens
        return n

    def schedule(self) -> StepPlan:
        want_prefill = self.prefill_pending()
        ready = any(q.prefilled for q in self.running)
        mix = want_prefill and ready and self.cfg.mixed_prefill_tokens > 0
        if (mix and self._stalled < self.cfg.max_decode_stall_steps
                and self.prefill_backlog() > self.cfg.max_prefill_tokens):
            mix = False  # burst: prefill-only step, the decodes wait (bounded)
            self._stalled += 1
        elif ready:
            self._stalled = 0
        plan = StepPlan(is_prefill=False)
        if mix:  # reserve the decode rows' slots first: preemption here frees blocks for admission
            plan.decode = self._reserve_decode(plan)
            mix = bool(plan.decode)
        if want_prefill:
            # prefill: first the next chunks of partially prefilled sequences, then newly arrived
            # (or preempted) requests, within the step's token budget
            budget = self.cfg.max_prefill_tokens
            if mix:
                budget = min(budget, self.cfg.mixed_prefill_tokens)
            # (a sequence whose last chunk is in flight - pending_first - has nothing left to prefill
            # and cannot decode before its first token is read back)
            for seq in [q for q in self.running if not q.prefilled and not q.pending_first]:
                if budget <= 0:
                    break
                self._take_chunk(seq, budget, plan)
                budget -= seq.chunk
            while budget > 0 and self.waiting and len(self.running) < self.cfg.max_num_seqs:  # admitted join running
                seq = self.waiting[0]
                n = seq.num_tokens - self.blocks.cached_prefix_tokens(seq)  # tokens left to compute
                if n > budget and not self.cfg.chunked_prefill and plan.seqs:
                    break
                if self.admit_gate is not None and not self.admit_gate(seq, len(self.running) + 1):
                    break
                if not self.blocks.can_allocate(seq) or not self.blocks.allocate(seq):
                    break  # allocate() undoes its prefix matches on failure: seq stays queued
                self.waiting.popleft()
                seq.status = SeqStatus.RUNNING
                self.running.append(seq)
                self._take_chunk(seq, budget if self.cfg.chunked_prefill else n, plan)
                budget -= seq.chunk
            if plan.seqs:
                plan.is_prefill = True
                return plan
        # decode every running (fully prefilled) sequence
        rows = plan.decode if mix else self._reserve_decode(plan)
        return StepPlan(is_prefill=False, seqs=rows, preempted=plan.preempted)

    def _reserve_decode(self, plan: StepPlan) -> list[Sequence]:
        """Make room for one more token of every prefilled running sequence, preempting the
        youngest running sequence while the cache is short; returns the decode rows."""
        i = 0
        while i < len(self.running):
            seq = self.running[i]
            if not seq.prefilled or self.blocks.ensure_slot(seq):
                i += 1
                continue
            victim = self.running.pop()  # youngest
            self._preempt(victim)
            plan.preempted.append(victim)
            # retry the same index (the victim may have been this very sequence)
        return [q for q in self.running if q.prefilled]

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
