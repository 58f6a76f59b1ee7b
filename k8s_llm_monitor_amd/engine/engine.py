"""The in-process inference engine that replaces the reference's intended remote OpenAI call
(``internal/config/config.go:38-46,141-145``; prompt flow ``docs/metrics-usage-example.md:244-306``).

``LLMEngine`` is single-threaded and step-driven (schedule -> prefill|decode -> sample -> stop
checks).  ``EngineService`` runs it on a dedicated thread behind a request queue so HTTP handler
threads (``/api/v1/query``, ``/api/v1/analyze/pod-communication``) submit prompts and block on a
future - that is the continuous-batching queue of the north star: requests arriving while others
decode join the running batch at the next step.

Tensor parallelism: the TP leader (tp_rank 0, the process that serves HTTP) owns the scheduler
and broadcasts each step's inputs to the other TP ranks over the CPU gloo group (SURVEY.md
§2.12 C-6); every rank runs the identical forward (RCCL all-reduces inside), and sampling is
replicated (same logits, same RNG counter) so no token broadcast is needed.
"""
from __future__ import annotations

import os
import queue
import threading
import time
import uuid
from collections import deque
from concurrent.futures import Future
from dataclasses import dataclass, field
from typing import Optional, Union

import torch

from ..models.checkpoint import config_from_hf, load_checkpoint
from ..models.config import ModelConfig, get_config
from ..models.llama import CausalLM
from ..parallel.state import ParallelState, get_state, serving_timeouts
from ..parallel.step_bus import KIND_DECODE, KIND_PICKLE, KIND_STOP, bus_slot_bytes, decode_message, make_step_bus
from ..parallel.health import PeerMonitor, gather_identities
from .block_manager import BlockManager
from .runner import ModelRunner, RunnerConfig
from .scheduler import Scheduler, SchedulerConfig
from .sequence import SamplingParams, Sequence, SeqStatus
from .tokenizer import tokenizer_for, tokenizer_from_dir


@dataclass
class EngineConfig:
    model: str = "llama-3-8b"
    max_num_seqs: int = 64
    max_model_len: int = 8192
    max_prefill_tokens: int = 16384
    chunked_prefill: bool = True  # prompts beyond a step's token budget prefill in chunks (scheduler.py)
    # prefill budget of a mixed prefill+decode step (scheduler.py); 0 = prefill steps stall decodes
    mixed_prefill_tokens: int = 16384
    # burst policy (scheduler.py): at most this many prefill-only steps in a row while decodes wait
    # and the prefill backlog exceeds one step; 0 = always mix.  K8SLLM_DECODE_STALL_STEPS
    max_decode_stall_steps: int = field(default_factory=lambda: int(os.environ.get("K8SLLM_DECODE_STALL_STEPS", "8")))
    kv_cache_gb: float = 32.0
    num_blocks: Optional[int] = None
    use_graphs: bool = True
    seed: int = 0
    tp_size: int = 1
    pipeline: bool = True  # overlap the host's per-step work with the GPU's decode step
    # reuse KV blocks of identical prompt prefixes (block_manager.py); K8SLLM_PREFIX_CACHE=0 disables
    prefix_caching: bool = field(default_factory=lambda: os.environ.get("K8SLLM_PREFIX_CACHE", "1") != "0")
    dtype: str = "bfloat16"  # compute / weight dtype ("float32" for CPU parity tests)
    # admission coalescing: when an idle engine receives a request, keep collecting arrivals until
    # none comes for `admit_gap_ms` (at most `admit_window_ms`) before the first prefill, so a
    # burst of queries starts as one full prefill batch instead of a lone first prompt
    admit_gap_ms: float = 2.0
    admit_window_ms: float = 20.0
    model_overrides: dict = field(default_factory=dict)
    # a Hugging Face model directory (config.json, *.safetensors, optional tokenizer.json): real
    # weights instead of the seeded random init (models/checkpoint.py); None = random init
    weights: Optional[str] = None


class _View:
    """What the runner needs of a sequence; built on non-leader TP ranks from the broadcast."""

    __slots__ = ("all_ids", "num_tokens", "block_table", "last_token", "params", "num_computed", "chunk",
                 "chunk_ids")

    def __init__(self, all_ids, num_tokens, block_table, last_token, params, num_computed=0, chunk=0,
                 chunk_ids=None):
        self.all_ids, self.num_tokens, self.block_table = all_ids, num_tokens, block_table
        self.last_token, self.params = last_token, params
        self.num_computed, self.chunk = num_computed, chunk
        self.chunk_ids = chunk_ids


class LLMEngine:
    def __init__(self, cfg: EngineConfig, device: Optional[Union[str, torch.device]] = None,
                 pstate: Optional[ParallelState] = None, model_cfg: Optional[ModelConfig] = None):
        self.cfg = cfg
        self.ps = pstate or get_state()
        if device is None:
            device = self.ps.device if self.ps.device.type == "cuda" else (
                "cuda" if torch.cuda.is_available() else "cpu")
        self.device = torch.device(device)
        if model_cfg is None and cfg.weights:
            model_cfg = config_from_hf(cfg.weights)
        mc = model_cfg or get_config(cfg.model)
        if cfg.model_overrides:
            mc = mc.replace(**cfg.model_overrides)
        self.model_cfg = mc
        t0 = time.perf_counter()
        self.model = CausalLM(mc, device=self.device, dtype=getattr(torch, cfg.dtype), seed=cfg.seed, pstate=self.ps,
                              init="empty" if cfg.weights else "random")
        if cfg.weights:
            load_checkpoint(self.model, cfg.weights)
        self.runner = ModelRunner(self.model, RunnerConfig(
            max_num_seqs=cfg.max_num_seqs, max_model_len=cfg.max_model_len, kv_cache_gb=cfg.kv_cache_gb,
            num_blocks=cfg.num_blocks, use_graphs=cfg.use_graphs, seed=cfg.seed))
        self.blocks = BlockManager(self.runner.num_blocks, prefix_caching=cfg.prefix_caching)
        self.sched = Scheduler(SchedulerConfig(max_num_seqs=cfg.max_num_seqs,
                                               max_prefill_tokens=cfg.max_prefill_tokens,
                                               max_model_len=self.runner.max_len,
                                               chunked_prefill=cfg.chunked_prefill,
                                               mixed_prefill_tokens=cfg.mixed_prefill_tokens,
                                               max_decode_stall_steps=cfg.max_decode_stall_steps), self.blocks)
        self.tokenizer = tokenizer_from_dir(cfg.weights, mc) if cfg.weights else tokenizer_for(mc)
        self.eos = set(mc.eos_ids)
        self.init_s = time.perf_counter() - t0
        self.counters = {"requests": 0, "finished": 0, "prompt_tokens": 0, "generated_tokens": 0,
                         "prefill_steps": 0, "decode_steps": 0, "mixed_steps": 0, "preemptions": 0,
                         "deadline_stops": 0, "step_failures": 0}
        self.is_leader = self.ps.tp_rank == 0
        self._inflight = None  # (seqs, DecodeHandle) of the enqueued, not yet read back decode step
        # (plan, DecodeHandle, step id) of the enqueued, not yet read back prefill-only step
        self._pf_inflight = None
        self._pf_step_id = 0
        self.trace: Optional[list] = [] if os.environ.get("K8SLLM_TRACE") else None  # (t, kind, n, tokens)
        self._inflight_rows: dict = {}
        # (rows, GPU ms) of decode steps that ran back to back, measured by events (the admission
        # model's samples: no host time, keyed by the step that actually ran)
        self.step_samples: deque = deque(maxlen=256)
        # TP: the step bus to the workers (shared-memory ring, parallel/step_bus.py) - collective
        self.bus = make_step_bus(self.ps, bus_slot_bytes(cfg.max_num_seqs, self.runner.max_len,
                                                         self.runner.max_blocks_per_seq)) if self.ps.tp_size > 1 else None
        self._publish = self.bus.send_raw if (self.bus is not None and self.is_leader) else None
        # TP: every rank's (pid, start time, host) - the leader's PeerMonitor watches its workers,
        # a worker checks it can see its leader (parallel/health.py)
        self.peer_idents = gather_identities(self.ps) if self.ps.tp_size > 1 else []
        if self.bus is not None and not self.is_leader:
            self.bus.set_leader(self.peer_idents[0])
        # custom all-reduce health: its error flag is copied back after every decode launch
        car = self.ps.custom_ar
        self._car_flag = None
        if car is not None and self.device.type == "cuda":
            self._car_flag = torch.zeros(1, dtype=torch.int32, pin_memory=True)
            self.runner.on_launched = lambda: car.error_async(self._car_flag)

    # ----------------------------------------------------------------- public API
    def warmup(self) -> None:
        """Capture the decode hipGraphs (all buckets); then the TP groups take their serving
        timeout (start-up is over: parallel/state.serving_timeouts)."""
        t0 = time.perf_counter()
        self.runner.capture_graphs()
        self.graph_s = time.perf_counter() - t0
        serving_timeouts(self.ps)

    def add_request(self, prompt: Union[str, list[int]], params: Optional[SamplingParams] = None,
                    request_id: Optional[str] = None, user=None, deadline: Optional[float] = None) -> Sequence:
        """``deadline`` (time.perf_counter clock): the sequence stops with finish_reason "deadline"
        at the first step resolved after it - an answer truncated to what fits the caller's time
        budget instead of work the caller has stopped waiting for."""
        ids = self.tokenizer.encode(prompt) if isinstance(prompt, str) else list(prompt)
        limit = self.runner.max_len - 1
        if len(ids) > limit - 1:  # keep room for at least one generated token; trim the middle
            keep = limit - 1
            ids = ids[: keep // 2] + ids[len(ids) - (keep - keep // 2):]
        seq = Sequence(prompt_ids=ids, params=params or SamplingParams(),
                       request_id=request_id or uuid.uuid4().hex[:16], user=user, deadline=deadline)
        self.sched.add(seq)
        if self.trace is not None:
            self.trace.append((time.perf_counter(), "add", 1, len(ids)))
        self.counters["requests"] += 1
        self.counters["prompt_tokens"] += len(ids)
        return seq

    def has_work(self) -> bool:
        return self.sched.has_work() or self._inflight is not None or self._pf_inflight is not None

    PENDING = -1  # placeholder for a token sampled by the in-flight decode step
    # tests install a callable(kind) here to inject faults into worker_loop (tests/test_tp_failure.py)
    worker_step_hook = None

    def step(self) -> list[Sequence]:
        """One engine step; returns the sequences that finished.

        Pipelined decode (``EngineConfig.pipeline``): a decode step is enqueued on the GPU before the
        previous one's tokens are read back, and each row whose input is such a not-yet-read token
        takes it from the device (``ModelRunner.decode_launch`` ``src_rows``).  The host's per-step
        work (scheduling, block bookkeeping, staging, stop checks, HTTP completions) then overlaps
        the GPU's step instead of sitting between steps.  A sequence that stops on EOS therefore
        runs one extra (discarded) step; length stops are predicted and never overrun.  Prefill
        steps resolve the in-flight decode first (they change the batch)."""
        if not self.cfg.pipeline:
            return self._step_sync()
        done: list[Sequence] = []
        s = self.sched
        if self._inflight is not None and (not s.running or s.prefill_pending()):
            done += self._resolve()
        plan = s.schedule()
        self.counters["preemptions"] += len(plan.preempted)
        if self._pf_inflight is not None:
            if plan.is_prefill and not plan.decode:
                # pipelined prefill: enqueue this step behind the in-flight one, then read that one
                # back - the host's scheduling and input staging overlap the GPU's previous step
                h = self._launch_prefill(plan)
                done += self._resolve_prefill()
                self._pf_inflight = h
                return done
            done += self._resolve_prefill()
            if not plan.is_prefill:
                # the decode rows left out the sequences whose first token was in flight: plan again
                plan = s.schedule()
                self.counters["preemptions"] += len(plan.preempted)
        if plan.empty:
            if self._inflight is not None:
                done += self._resolve()
            return done
        if plan.is_prefill:
            if not plan.decode and self._inflight is None:
                self._pf_inflight = self._launch_prefill(plan)  # read back by the next step
                return done
            return done + self._run_sync(plan)
        # length-limited sequences whose last token is already in flight stop on resolve: skip them
        seqs = [q for q in plan.seqs if not self._length_done(q)]
        if not seqs:
            return done + (self._resolve() if self._inflight is not None else [])
        seqs = self._attention_row_order(seqs)
        prev_rows = self._inflight_rows
        src = [prev_rows.get(q.seq_id, -1) for q in seqs]
        t_l = time.perf_counter() if self.trace is not None else 0.0
        handle = self.runner.decode_launch(seqs, src, publish=self._publish)
        self.counters["decode_steps"] += 1
        if self.trace is not None:
            now = time.perf_counter()
            self.trace.append((now, "decode", len(seqs), 0))
            self.trace.append((now, "dlaunch", len(seqs), (now - t_l) * 1e3))  # host ms in decode_launch
        for q in seqs:
            q.output_ids.append(self.PENDING)
        prev = self._inflight
        self._inflight = (seqs, handle)
        self._inflight_rows = {q.seq_id: i for i, q in enumerate(seqs)}
        if prev is not None:
            done += self._resolve_step(*prev)
        return done

    def _attention_row_order(self, seqs: list) -> list:
        """Decode batch rows ordered for the paged-attention grid (one workgroup per (row, kv head),
        two per CU): with a 64-row graph every XCD runs the 64 rows of one kv head and workgroups z
        and z + 32 share a CU, so rows 0..31 take the 32 longest contexts (longest first) and rows
        32..63 the rest shortest first - each CU gets one long and one short sequence and no CU
        keeps two long ones running after the rest drained (ragged 1.3k-2.3k contexts: 72.7 vs
        77.1 us per layer for an arbitrary order, profiles/r03/decode_row_order.jsonl).  Other
        bucket sizes: longest first (74.6 us).  Row order is free: each row's input token is
        located through ``src`` and every per-row result is keyed by the sequence.
        ``_ROW_ORDER = False`` keeps the scheduler's order."""
        if not _ROW_ORDER or len(seqs) < 2:
            return seqs
        srt = sorted(seqs, key=lambda q: -q.num_tokens)
        n = len(srt)
        b = self.runner.bucket_for(n) if self.runner.graphs else n
        half = b // 2
        if b != 2 * _CUS_PER_XCD or n <= half:
            return srt
        return srt[:half] + srt[half:][::-1]

    def _launch_prefill(self, plan) -> tuple:
        """Enqueue a prefill-only step without reading its tokens back.  Chunk accounting happens
        now; a sequence whose prompt this step completes waits in ``pending_first`` (neither
        prefillable nor decodable) until :meth:`_resolve_prefill` appends its first token."""
        if self.bus is not None:
            self.bus.send_obj(self._pack(plan))
        plan.chunks = [q.chunk for q in plan.seqs]  # for the trace (chunk_done clears them)
        t_l = time.perf_counter() if self.trace is not None else 0.0
        h = self.runner.prefill_launch(plan.seqs)
        if self.trace is not None:  # host ms to stage and enqueue the step (exposed on a wave's first step)
            self.trace.append((time.perf_counter(), "plaunch", len(plan.seqs), (time.perf_counter() - t_l) * 1e3))
        self._pf_step_id += 1
        sid = self._pf_step_id
        for seq in plan.seqs:
            if self.sched.chunk_done(seq):
                seq.prefilled = False
                seq.pending_first = sid
        return plan, h, sid

    def _resolve_prefill(self) -> list[Sequence]:
        plan, h, sid = self._pf_inflight
        self._pf_inflight = None
        toks = self.runner.decode_collect(h)
        self._check_collectives()
        self.counters["prefill_steps"] += 1
        if self.trace is not None:
            self.trace.append((time.perf_counter(), "prefill", len(plan.seqs), sum(plan.chunks)))
        now = time.perf_counter()
        done = []
        for seq, tok in zip(plan.seqs, toks):
            if seq.pending_first != sid:
                continue  # a chunk short of the prompt's end, or freed (preempted / aborted) since
            seq.pending_first = 0
            seq.prefilled = True
            seq.output_ids.append(int(tok))
            self.counters["generated_tokens"] += 1
            if seq.t_first_token is None:
                seq.t_first_token = now
            reason = self._stop_reason(seq, int(tok), now=now)
            if reason:
                seq.t_finish = now
                self._finish(seq, reason)
                done.append(seq)
        return done

    def _length_done(self, q: Sequence) -> bool:
        return len(q.output_ids) >= q.params.max_tokens or q.num_tokens >= self.runner.max_len

    def _resolve(self) -> list[Sequence]:
        seqs, handle = self._inflight
        self._inflight = None
        self._inflight_rows = {}
        return self._resolve_step(seqs, handle)

    def _check_collectives(self) -> None:
        if self._car_flag is not None and int(self._car_flag[0]) != 0:
            raise RuntimeError("custom all-reduce: a TP peer did not arrive (step output invalid)")

    def _resolve_step(self, seqs: list, handle) -> list[Sequence]:
        t_w = time.perf_counter() if self.trace is not None else 0.0
        toks = self.runner.decode_collect(handle)
        if self.trace is not None:  # host ms blocked on the step's tokens (0: the host is the bottleneck)
            self.trace.append((time.perf_counter(), "dwait", len(seqs), (time.perf_counter() - t_w) * 1e3))
        self._check_collectives()
        ms = handle.gpu_ms() if hasattr(handle, "gpu_ms") else None
        if ms is not None:  # a back-to-back decode step: its GPU time at this row count and context
            self.step_samples.append((len(seqs), ms, sum(q.num_tokens for q in seqs)))
        now = time.perf_counter()
        done = []
        for q, tok in zip(seqs, toks):
            if q.status in (SeqStatus.FINISHED, SeqStatus.ABORTED):
                continue  # stopped on the previous step; this step's token is discarded
            tok = int(tok)
            out = q.output_ids
            i = len(out) - 1  # placeholders trail the answer (at most two steps in flight): O(1)
            while i > 0 and out[i - 1] == self.PENDING:
                i -= 1
            out[i] = tok
            self.counters["generated_tokens"] += 1
            if q.t_first_token is None:
                q.t_first_token = now
            reason = self._stop_reason(q, tok, n_out=i + 1, now=now)
            if reason:
                del q.output_ids[i + 1:]  # drop the token of a step launched past the stop
                q.t_finish = now
                self._finish(q, reason)
                done.append(q)
        return done

    def _finish(self, q: Sequence, reason: str) -> None:
        if q.status == SeqStatus.WAITING:  # preempted while its last token was in flight
            try:
                self.sched.waiting.remove(q)
            except ValueError:
                pass
        self.sched.finish(q, reason)
        self.counters["finished"] += 1

    def _step_sync(self) -> list[Sequence]:
        plan = self.sched.schedule()
        self.counters["preemptions"] += len(plan.preempted)
        if plan.empty:
            return []
        return self._run_sync(plan)

    def _run_sync(self, plan) -> list[Sequence]:
        if self.bus is not None and plan.is_prefill:
            self.bus.send_obj(self._pack(plan))
        if plan.is_prefill:
            toks = self.runner.prefill(plan.seqs, plan.decode)
            self._check_collectives()  # prefill / mixed steps route small all-reduces through custom AR too
            self.counters["prefill_steps"] += 1
            if plan.decode:
                self.counters["mixed_steps"] += 1
            if self.trace is not None:
                self.trace.append((time.perf_counter(), "prefill", len(plan.seqs),
                                   sum(q.chunk for q in plan.seqs)))
            rows = list(plan.decode) + list(plan.seqs)
            nd = len(plan.decode)
        else:
            toks = self.runner.decode(plan.seqs, publish=self._publish)
            self._check_collectives()
            self.counters["decode_steps"] += 1
            rows, nd = plan.seqs, len(plan.seqs)
        now = time.perf_counter()
        done = []
        for i, (seq, tok) in enumerate(zip(rows, toks)):
            if i >= nd and not self.sched.chunk_done(seq):
                continue  # a chunk short of the prompt's end: no token yet
            seq.output_ids.append(int(tok))
            self.counters["generated_tokens"] += 1
            if seq.t_first_token is None:
                seq.t_first_token = now
            reason = self._stop_reason(seq, int(tok), now=now)
            if reason:
                seq.t_finish = now
                self._finish(seq, reason)
                done.append(seq)
        return done

    def _stop_reason(self, seq: Sequence, tok: int, n_out: Optional[int] = None,
                     now: Optional[float] = None) -> Optional[str]:
        p = seq.params
        n = len(seq.output_ids) if n_out is None else n_out
        if not p.ignore_eos and (tok in self.eos or tok in p.stop_token_ids):
            return "stop"
        if n >= p.max_tokens:
            return "length"
        if len(seq.prompt_ids) + n >= self.runner.max_len:
            return "length"
        if seq.deadline is not None and now is not None and now >= seq.deadline:
            self.counters["deadline_stops"] += 1
            return "deadline"
        return None

    def abort(self, seq: Sequence) -> None:
        self.sched.abort(seq)

    def reset(self) -> list[Sequence]:
        """After a failed step: drop the in-flight decode and abort every running and waiting
        sequence (their KV blocks return to the pool).  Returns the aborted sequences."""
        self._inflight = None
        self._inflight_rows = {}
        self._pf_inflight = None
        if self.device.type == "cuda":
            try:
                torch.cuda.synchronize(self.device)
            except Exception:  # noqa: BLE001 - a sticky device error: the blocks are still freed
                pass
        seqs = list(self.sched.running) + list(self.sched.waiting)
        for q in seqs:
            self.sched.abort(q)
        return seqs

    def generate(self, prompts: list, params: Optional[SamplingParams] = None) -> list[Sequence]:
        seqs = [self.add_request(p, params) for p in prompts]
        while any(s.status not in (SeqStatus.FINISHED, SeqStatus.ABORTED) for s in seqs):
            self.step()
        return seqs

    def has_inflight(self) -> bool:
        return self._inflight is not None

    def decode_text(self, seq: Sequence) -> str:
        return self.tokenizer.decode(seq.output_ids)

    def stats(self) -> dict:
        d = dict(self.counters)
        d.update(self.sched.stats())
        d.update({"model": self.model_cfg.name, "tp_size": self.ps.tp_size, "device": str(self.device),
                  "graph_buckets": sorted(self.runner.graphs), "max_num_seqs": self.cfg.max_num_seqs})
        return d

    # ----------------------------------------------------------------- tensor parallel
    @staticmethod
    def _pack(plan) -> tuple:
        """A prefill / mixed step for the TP workers: each chunk's token ids (not the whole prompt)
        and block table, and the decode rows of a mixed step."""
        return ([(s.all_ids[s.num_computed:s.num_computed + s.chunk], s.block_table, _params_t(s.params),
                  s.num_computed, s.chunk) for s in plan.seqs],
                [(s.last_token, s.num_tokens, s.block_table, _params_t(s.params)) for s in plan.decode])

    def worker_loop(self) -> None:
        """Non-leader TP ranks: mirror the leader's steps (step bus) until it sends STOP."""
        pending = None
        while True:
            kind, payload = decode_message(self.bus.recv())
            if self.worker_step_hook is not None:  # fault injection (tests only; None in production)
                self.worker_step_hook(kind)
            if kind == KIND_DECODE:
                h = self.runner.decode_launch_raw(*payload)
                if pending is not None:  # keep at most two steps enqueued (staging is double-buffered)
                    self.runner.decode_collect(pending)
                    self._check_collectives()
                pending = h
                continue
            if pending is not None:
                self.runner.decode_collect(pending)
                self._check_collectives()
                pending = None
            if kind == KIND_STOP:
                return
            if kind == KIND_PICKLE:
                items, dec = payload
                views = [_View(None, nc + ch, bt, None, SamplingParams(*p), nc, ch, chunk_ids=ids)
                         for ids, bt, p, nc, ch in items]
                dviews = [_View(None, n, bt, last, SamplingParams(*p)) for last, n, bt, p in dec]
                self.runner.prefill(views, dviews)
                self._check_collectives()

    def stop_workers(self) -> None:
        if self._inflight is not None:
            self._resolve()
        if self.bus is not None and self.is_leader:
            self.bus.send_stop()


def _params_t(p: SamplingParams) -> tuple:
    return (p.max_tokens, p.temperature, p.top_k, p.top_p, p.ignore_eos, tuple(p.stop_token_ids))


class _Skip(Exception):
    pass


class TpotModel:
    """Decode step time (ms) learned online from measured steps.

    Two models, the richer one used once it is trustworthy:

    * by batch size - an EWMA per batch size seen and a least-squares line t(b) = a + c*b over
      those sizes; with one size seen, that time is used for every size up to it and grows in
      proportion beyond it;
    * by batch size AND context - t(b, kv) = a + r*b + k*kv with kv the batch's total context
      tokens (every decode step streams the weights once - a - and each cached token's K/V once -
      k; r is the per-row activation / sampling cost), a non-negative least-squares fit over the
      last ``window`` (b, kv, ms) samples, refit every ``refit`` new samples and used only when it
      explains the samples to within ``max_rel_err`` (RMS).  Attention time grows with every
      generated token, so a batch-size-only EWMA, which follows the latest (longest-context) steps,
      overstates the step time of an answer that starts now - the admission gate would refuse
      answers that fit (profiles/r04/production_2000tok_b64.json: predicted 6.66 ms at 40 rows,
      5.91 ms measured over the answers).
    """

    def __init__(self, alpha: float = 0.25, window: int = 1024, refit: int = 64, min_samples: int = 48,
                 max_rel_err: float = 0.08):
        self.alpha = alpha
        self.ew: dict[int, float] = {}
        self._fit: Optional[tuple] = None
        self.samples: deque = deque(maxlen=window)  # (b, kv tokens, ms)
        self.refit, self.min_samples, self.max_rel_err = refit, min_samples, max_rel_err
        self._since = 0
        self.kv_fit: Optional[tuple] = None  # (a, r, k per 1000 tokens, rms rel err)

    def record(self, b: int, ms: float, kv: Optional[int] = None) -> None:
        if b <= 0 or ms <= 0:
            return
        old = self.ew.get(b)
        self.ew[b] = ms if old is None else (1 - self.alpha) * old + self.alpha * ms
        self._fit = None
        if kv is not None and kv > 0:
            self.samples.append((b, kv, ms))
            self._since += 1
            if len(self.samples) >= self.min_samples and (self.kv_fit is None or self._since >= self.refit):
                self._fit_kv()

    def _fit_kv(self) -> None:
        import numpy as np

        self._since = 0
        a = np.asarray(self.samples, dtype=np.float64)
        X = np.stack([np.ones(len(a)), a[:, 0], a[:, 1] / 1000.0], 1)
        y = a[:, 2]
        if np.ptp(X[:, 2]) <= 0.05 * max(1.0, X[:, 2].mean()):
            return  # no context spread: the slope is not identifiable
        # one batch size only: the per-row term is not separable from the constant - leave it out
        active = [0, 1, 2] if np.ptp(X[:, 1]) > 0 else [0, 2]
        coef = np.zeros(3)
        for _ in range(3):  # non-negative least squares by dropping negative terms (3 unknowns)
            sol, *_ = np.linalg.lstsq(X[:, active], y, rcond=None)
            if (sol >= 0).all():
                coef[:] = 0.0
                coef[active] = sol
                break
            active = [c for c, v in zip(active, sol) if v > 0] or [0]
        else:
            return
        err = float(np.sqrt(np.mean(((X @ coef) - y) ** 2 / y ** 2)))
        self.kv_fit = (float(coef[0]), float(coef[1]), float(coef[2]), err) if err <= self.max_rel_err else None

    def estimate(self, b: int, kv: Optional[float] = None) -> Optional[float]:
        if not self.ew:
            return None
        b = max(1, b)
        if kv is not None and self.kv_fit is not None:
            a, r, k, _ = self.kv_fit
            return max(0.5 * min(self.ew.values()), a + r * b + k * kv / 1000.0)
        if len(self.ew) == 1:
            (b0, t0), = self.ew.items()
            return t0 if b <= b0 else t0 * b / b0
        if self._fit is None:
            xs, ys = list(self.ew), list(self.ew.values())
            n = len(xs)
            mx, my = sum(xs) / n, sum(ys) / n
            vx = sum((x - mx) ** 2 for x in xs)
            c = max(0.0, sum((x - mx) * (y - my) for x, y in zip(xs, ys)) / vx) if vx > 0 else 0.0
            self._fit = (my - c * mx, c, min(ys))
        a, c, lo = self._fit
        return max(lo, a + c * b)

    def snapshot(self) -> dict:
        d = {str(b): round(t, 3) for b, t in sorted(self.ew.items())}
        if self.kv_fit is not None:
            a, r, k, e = self.kv_fit
            d["kv_fit"] = {"ms_const": round(a, 4), "ms_per_row": round(r, 5), "ms_per_1k_ctx_tokens": round(k, 5),
                           "rms_rel_err": round(e, 4), "samples": len(self.samples)}
        return d


_ROW_ORDER = True  # decode rows paired long / short per CU (tests may turn it off)
_CUS_PER_XCD = 32  # MI355X: 256 CUs in 8 XCDs


class AnswerLengths:
    """Observed answer lengths (generated tokens) of requests that stop on EOS / stop tokens or at
    their max_tokens, for the deadline admission: an answer that may stop early is budgeted at the
    ``q``-quantile of recent answers instead of its max_tokens (requests with ``ignore_eos``
    always run to max_tokens and are budgeted so)."""

    def __init__(self, keep: int = 512, min_samples: int = 16, q: float = 0.9):
        self.lens: deque = deque(maxlen=keep)
        self.min_samples, self.q = min_samples, q
        self._cached: Optional[int] = None

    def record(self, n: int) -> None:
        self.lens.append(int(n))
        self._cached = None

    def quantile(self) -> Optional[int]:
        if len(self.lens) < self.min_samples:
            return None
        if self._cached is None:
            xs = sorted(self.lens)
            self._cached = xs[min(len(xs) - 1, int(len(xs) * self.q))]
        return self._cached


class EngineOverloaded(RuntimeError):
    """Admission refused: the queue is full or the request cannot start within its deadline
    (the HTTP layer answers 503 - SURVEY.md §5 failure detection: reject, never crash or hang)."""


class EngineUnavailable(RuntimeError):
    """The engine is unhealthy (repeated step failures) and accepts no work (HTTP 503)."""


class EngineService:
    """Runs an LLMEngine on its own thread; thread-safe ``submit`` returns a Future that resolves
    to ``(text, sequence)``.

    Serving robustness:
    * bounded admission - at most ``max_queue`` requests wait (queued + scheduler-waiting); beyond
      that, and for a request whose estimated time to first token already exceeds its deadline,
      ``submit`` fails the future with EngineOverloaded at once;
    * deadlines - ``submit(deadline=...)`` stops the sequence at the deadline with finish_reason
      "deadline" (a truncated answer, KV freed), and a request still waiting when its deadline
      passes is dropped with EngineOverloaded;
    * deadline-feasible admission - a waiting request with a deadline starts only when the learned
      decode step time at the batch it would join (TpotModel, fed by GPU-event step times) x its
      expected answer length (max_tokens with ignore_eos, else at most the observed 90th-percentile
      answer length: AnswerLengths), plus its prefill, fits its deadline AND every running
      request's expected remaining tokens still fit theirs (a preempted sequence resumes without
      the gate; a request without a deadline is not held back by the running ones); a request
      that cannot finish in time even once the first running answer completes is refused at once
      (EngineOverloaded -> 503) instead of being truncated later (reference budget:
      cmd/server/main.go:147-148 15 s write timeout, internal/config/config.go:145 llm.timeout);
    * cancellation - ``cancel(fut)`` aborts the sequence and frees its KV blocks before the next
      step;
    * step failures - an exception inside a step fails only the requests in flight, resets the
      engine's batch and keeps serving; ``max_failures`` failures within ``failure_window_s`` (or
      any failure at TP > 1, where the workers' mirrored state is unknown) mark the service
      unhealthy: ``healthy`` turns False and every later submit fails with EngineUnavailable;
    * failure detection (parallel/health.py) - a watchdog thread marks the service unhealthy when a
      step stays in flight longer than ``watchdog_s`` (a collective that never completes), and at
      TP > 1 the leader's PeerMonitor does so as soon as a worker process is gone; both fail every
      request in flight or queued at once (EngineUnavailable -> 503) and turn /health to 503,
      instead of the leader blocking until the process-group timeout behind a 200 /health.
    """

    def __init__(self, engine: LLMEngine, max_queue: Optional[int] = None, max_failures: int = 3,
                 failure_window_s: float = 60.0, watchdog_s: Optional[float] = None):
        """``watchdog_s``: a step still in flight after this long marks the service unhealthy
        (default ``K8SLLM_STEP_WATCHDOG_S``, else 30 s = twice the reference's 15 s write timeout
        at TP > 1 on the GPU - a decode step takes milliseconds, a prefill step well under a
        second - and off otherwise; 0 disables)."""
        self.engine = engine
        self.max_queue = max_queue if max_queue is not None else 4 * engine.cfg.max_num_seqs
        self.max_failures, self.failure_window_s = max_failures, failure_window_s
        self._q: queue.Queue = queue.Queue()
        self._stop = threading.Event()
        self._thread = threading.Thread(target=self._loop, name="llm-engine", daemon=True)
        self._lock = threading.Lock()
        self._error: Optional[BaseException] = None
        self._failures: deque = deque()
        self.latencies_ms: deque = deque(maxlen=4096)
        self._streams: dict = {}  # seq_id -> [seq, tokens delivered, on_tokens]
        self._cancels: queue.SimpleQueue = queue.SimpleQueue()  # futures whose requests to abort
        self.cancelled = 0
        self.rejected = 0
        self.expired = 0
        # prefill throughput estimate (tokens/s, EWMA over prefill steps) for deadline admission
        self._prefill_tps: Optional[float] = None
        self._waiting_est = 0  # prompt tokens waiting in the scheduler (engine thread writes)
        self.tpot = TpotModel()
        self.answer_lens = AnswerLengths()
        self._step_cache: dict = {}  # per-step memo of the running set's deadline slack
        self.deadline_margin = 1.05  # safety factor on the estimated completion time
        self.infeasible = 0  # refused because the answer could not finish before its deadline
        self._gpu_tpot = False  # step times come from GPU events (ModelRunner._chain_event)
        engine.sched.admit_gate = self._admit_ok
        # failure detection (parallel/health.py): step watchdog + TP worker liveness
        # (default on only for TP > 1 on the GPU, where a wedged collective is what it catches; at
        # TP = 1 or on the CPU a legitimately slow step must not 503 the service for good)
        if watchdog_s is None:
            env = os.environ.get("K8SLLM_STEP_WATCHDOG_S")
            watchdog_s = float(env) if env else (30.0 if engine.ps.tp_size > 1 and engine.device.type == "cuda" else 0.0)
        self.watchdog_s = watchdog_s
        self._step_t0: Optional[float] = None  # monotonic start of the step in flight
        self.peer_monitor = None
        if engine.ps.tp_size > 1 and engine.is_leader and engine.peer_idents:
            peers = {r: ident for r, ident in enumerate(engine.peer_idents) if r != engine.ps.tp_rank}
            self.peer_monitor = PeerMonitor(
                peers, lambda r, ident: self._declare_dead(EngineUnavailable(
                    f"TP worker rank {r} (pid {ident[0]}) exited: the group cannot run another step")))
        self._wd_stop = threading.Event()
        self._watchdog = threading.Thread(target=self._watch, name="llm-engine-watchdog", daemon=True)
        self._thread.start()
        self._watchdog.start()

    def _watch(self) -> None:
        while not self._wd_stop.wait(0.25):
            t0 = self._step_t0
            if (self._error is None and t0 is not None and self.watchdog_s > 0
                    and time.monotonic() - t0 > self.watchdog_s):
                self._declare_dead(EngineUnavailable(
                    f"engine step in flight for more than {self.watchdog_s:.0f} s (a TP collective is not completing)"))
            if self._error is not None:
                return

    def _declare_dead(self, e: BaseException) -> None:
        """Mark the service unhealthy from a monitor thread (the engine thread may be blocked inside
        a collective and never return): /health turns 503 and every request in flight or queued
        fails now with EngineUnavailable instead of waiting for the process-group timeout."""
        import logging

        with self._lock:
            if self._error is not None:
                return
            self._error = e
        logging.getLogger("engine").error("engine unhealthy: %s", e)
        err = e if isinstance(e, EngineUnavailable) else EngineUnavailable(str(e))
        futs = []
        try:
            futs += [q.user for q in list(self.engine.sched.running) + list(self.engine.sched.waiting)]
        except Exception:  # noqa: BLE001 - lists mutating under a live engine thread: best effort
            pass
        while True:
            try:
                futs.append(self._q.get_nowait()[3])
            except queue.Empty:
                break
        for f in futs:
            if isinstance(f, Future) and not f.done():
                try:
                    f.set_exception(err)
                except Exception:  # noqa: BLE001 - resolved concurrently by the engine thread
                    pass

    @property
    def healthy(self) -> bool:
        return self._error is None and self._thread.is_alive()

    def pending(self) -> int:
        """Requests admitted but not yet running (HTTP queue + scheduler waiting list)."""
        return self._q.qsize() + len(self.engine.sched.waiting)

    def submit(self, prompt: Union[str, list[int]], params: Optional[SamplingParams] = None,
               request_id: Optional[str] = None, on_tokens=None, deadline: Optional[float] = None) -> Future:
        """``on_tokens(ids)`` (optional, streaming): called on the engine thread with each batch of
        newly generated token ids, before the future resolves; keep it cheap (e.g. a queue put).
        ``deadline``: time.perf_counter() value by which the answer is due (see class docstring)."""
        fut: Future = Future()
        if not self.healthy:
            fut.set_exception(EngineUnavailable(f"engine unhealthy: {self._error!r}"))
            return fut
        if isinstance(prompt, str):
            # tokenize on the caller's thread: the native BPE releases the GIL, so a burst's HTTP
            # handler threads encode in parallel instead of the engine thread encoding the whole
            # burst serially while the GPU waits for the first prefill
            try:
                prompt = self.engine.tokenizer.encode(prompt)
            except Exception as e:  # noqa: BLE001 - reject this request only
                fut.set_exception(e)
                return fut
        if self.pending() >= self.max_queue:
            self.rejected += 1
            fut.set_exception(EngineOverloaded(f"request queue full ({self.max_queue} waiting)"))
            return fut
        if deadline is not None and self._prefill_tps:
            # queued prompt tokens ahead of this one at the measured prefill rate: if even the first
            # token cannot arrive before the deadline, say so now instead of timing out later
            ahead = self._waiting_est + self._q.qsize() * 1024
            if time.perf_counter() + ahead / self._prefill_tps > deadline:
                self.rejected += 1
                fut.set_exception(EngineOverloaded("estimated time to first token exceeds the deadline"))
                return fut
        tr = self.engine.trace
        if tr is not None:
            tr.append((time.perf_counter(), "submit", 1, 0))
        self._q.put((prompt, params, request_id, fut, on_tokens, deadline))
        return fut

    def cancel(self, fut: Future) -> bool:
        """Abort the request behind ``fut`` (e.g. its streaming client disconnected or its caller
        timed out): the future is cancelled at once; the engine thread drops the sequence and frees
        its KV blocks before its next step.  False if the answer was already complete."""
        if not fut.cancel():
            return False
        self._cancels.put(fut)
        return True

    def _apply_cancels(self) -> None:
        eng = self.engine
        futs = set()
        while True:
            try:
                futs.add(self._cancels.get_nowait())
            except queue.Empty:
                break
        for s in list(eng.sched.running) + list(eng.sched.waiting):
            if s.user in futs:
                eng.abort(s)
                self._streams.pop(s.seq_id, None)
                self.cancelled += 1

    def _prefill_s(self, seq: Sequence) -> float:
        return (seq.num_tokens / self._prefill_tps) if self._prefill_tps else 0.0

    def _expected_rem(self, seq: Sequence) -> int:
        """Tokens ``seq`` is expected to still generate: its max_tokens minus what it already has
        (a preempted sequence keeps its answer so far), or - when it may stop on EOS - at most the
        observed 90th-percentile answer length (AnswerLengths) minus that."""
        gen = sum(1 for t in seq.output_ids if t >= 0)
        rem = max(0, seq.params.max_tokens - gen)
        if seq.params.ignore_eos:
            return rem
        q = self.answer_lens.quantile()
        if q is None:
            return rem
        return min(rem, max(q - gen, 32))

    def _kv_now(self) -> int:
        """Total context tokens of the running batch (memoised per engine step and batch size)."""
        key = ("kv", len(self.engine.sched.running))
        v = self._step_cache.get(key)
        if v is None:
            v = self._step_cache[key] = sum(q.num_tokens for q in self.engine.sched.running)
        return v

    def _backlog_s(self) -> float:
        """Seconds of prefill still owed to admitted sequences (prompt tokens not yet computed):
        in a burst every answer's first decode step waits for the whole burst's prefill, not only
        its own (production runs at 64 concurrent: ~0.9 s)."""
        if not self._prefill_tps:
            return 0.0
        key = ("backlog", len(self.engine.sched.running))
        v = self._step_cache.get(key)
        if v is None:
            v = self._step_cache[key] = sum(max(0, q.num_tokens - q.num_computed)
                                            for q in self.engine.sched.running) / self._prefill_tps
        return v

    def _answer_s(self, n: int, rem: int, extra_kv: int = 0) -> Optional[float]:
        """Seconds for ``rem`` more decode steps at batch ``n``, with the safety margin.  With the
        context-aware model the step time is taken at the batch's mean context over those steps:
        today's running contexts + ``extra_kv`` (a joiner's prompt) + n tokens per step, rem / 2
        steps on average (running answers are assumed not to finish earlier - conservative)."""
        kv = None
        if self.tpot.kv_fit is not None:
            kv = self._kv_now() + extra_kv + n * rem / 2.0
        t = self.tpot.estimate(n, kv)
        return None if t is None else rem * t * 1e-3 * self.deadline_margin

    def _running_slack(self, n_after: int, now: float, extra_kv: int = 0) -> float:
        """Smallest (deadline - expected finish) over the running requests that have a deadline, at
        batch ``n_after``; memoised per engine step (the gate and the infeasibility sweep of every
        waiting request reuse it; joiners' prompts are bucketed by 256 tokens)."""
        bucket = (extra_kv + 255) // 256
        key = ("slack", n_after, bucket, len(self.engine.sched.running))
        v = self._step_cache.get(key)
        if v is None:
            v = float("inf")
            for q in self.engine.sched.running:
                if q.deadline is not None:
                    t = self._answer_s(n_after, self._expected_rem(q), bucket * 256)
                    v = min(v, q.deadline - now - (t or 0.0))
            self._step_cache[key] = v
        return v

    def _admit_ok(self, seq: Sequence, n_after: int) -> bool:
        """Scheduler admission gate (engine thread): does ``seq`` finish before its deadline at the
        batch it would join, without pushing a running request past its own deadline?
        A preempted sequence (it already has answer tokens) resumes without the gate: it was
        admitted once, and refusing it would freeze admission behind it until its deadline.  A
        request without a deadline is not held back by the running requests' deadlines."""
        if seq.output_ids:
            return True
        if seq.deadline is None:
            return True
        ans = self._answer_s(n_after, self._expected_rem(seq), seq.num_tokens)
        if ans is None:
            return True
        now = time.perf_counter()
        pre, backlog = self._prefill_s(seq), self._backlog_s()
        if now + backlog + pre + ans > seq.deadline:
            return False
        return pre <= self._running_slack(n_after, now, seq.num_tokens) - backlog

    def _infeasible(self, seq: Sequence, now: float) -> bool:
        """A never-started request that cannot finish before its deadline even if it starts when
        the first running answer completes (or now, if the gate admits it now)."""
        running = self.engine.sched.running
        n = max(1, len(running))
        ans = self._answer_s(n, self._expected_rem(seq), seq.num_tokens)
        if ans is None or seq.deadline is None:
            return False
        wait = 0.0
        if not self._admit_ok(seq, len(running) + 1):
            key = ("minrem",)
            m = self._step_cache.get(key)
            if m is None:
                m = self._step_cache[key] = min((self._expected_rem(q) for q in running), default=0)
            wait = self._answer_s(n, m) or 0.0
        return now + max(wait, self._backlog_s()) + self._prefill_s(seq) + ans > seq.deadline

    def _expire_waiting(self) -> None:
        """Waiting requests whose deadline has passed: one that never started is dropped
        (EngineOverloaded, HTTP 503); a preempted one that already generated tokens ends with
        finish_reason "deadline" and its partial answer, like a running sequence at its deadline."""
        eng = self.engine
        now = time.perf_counter()
        for s in [s for s in eng.sched.waiting if s.deadline is not None and now >= s.deadline]:
            partial = [t for t in s.output_ids if t >= 0]
            if partial:
                s.output_ids[:] = partial
                s.t_finish = now
                eng.counters["deadline_stops"] += 1
                eng._finish(s, "deadline")
                if self._streams:
                    self._push_streams()
                if isinstance(s.user, Future) and not s.user.done():
                    self.latencies_ms.append(s.timings()["latency_ms"])
                    s.user.set_result((eng.decode_text(s), s))
                continue
            eng.abort(s)
            self._streams.pop(s.seq_id, None)
            self.expired += 1
            if isinstance(s.user, Future) and not s.user.done():
                s.user.set_exception(EngineOverloaded("request expired in the queue before it could start"))
        # never-started requests that can no longer finish in time: refuse now, not at the deadline
        for s in [s for s in eng.sched.waiting if s.deadline is not None and not s.output_ids
                  and self._infeasible(s, now)]:
            eng.abort(s)
            self._streams.pop(s.seq_id, None)
            self.infeasible += 1
            if isinstance(s.user, Future) and not s.user.done():
                s.user.set_exception(EngineOverloaded("the answer cannot finish before the deadline at the current load"))

    def _drain(self, block: bool, gather: bool = False) -> None:
        """Move queued requests into the engine.  ``block``: the engine is idle - wait for one.
        ``gather``: a full prefill step is running on the GPU and the next one is not full yet -
        keep collecting a burst's arrivals (the wait is hidden behind the running step) so the
        next pipelined prefill step is planned full, not with the part of the burst that happened
        to be queued (which left a partial step plus a tiny tail step per burst)."""
        cfg = self.engine.cfg
        try:
            if block:
                item = self._q.get(timeout=0.05)
            elif gather:
                item = self._q.get(timeout=cfg.admit_gap_ms * 1e-3)
            else:
                item = self._q.get_nowait()
        except queue.Empty:
            return
        # the engine was idle, or gathering: let a burst gather
        coalesce = (block or gather) and cfg.admit_window_ms > 0
        t_end = time.perf_counter() + cfg.admit_window_ms * 1e-3
        while item is not None:
            prompt, params, rid, fut, on_tokens, deadline = item
            try:
                if fut.cancelled():  # cancelled while queued
                    raise _Skip()
                seq = self.engine.add_request(prompt, params, rid, user=fut, deadline=deadline)
                if on_tokens is not None:
                    self._streams[seq.seq_id] = [seq, 0, on_tokens]
            except _Skip:
                pass
            except Exception as e:  # noqa: BLE001 - reject this request only
                fut.set_exception(e)
            if coalesce and self._waiting_tokens() >= cfg.max_prefill_tokens:
                # a full prefill step is queued: start it now - the rest of the burst is drained
                # while that step runs (draining it first held the launch until the burst ended)
                break
            try:
                item = self._q.get_nowait()
            except queue.Empty:
                item = None
                wait = min(cfg.admit_gap_ms * 1e-3, t_end - time.perf_counter()) if coalesce else 0.0
                if wait > 0:
                    try:
                        item = self._q.get(timeout=wait)
                    except queue.Empty:
                        item = None

    def _waiting_tokens(self) -> int:
        return sum(q.num_tokens for q in self.engine.sched.waiting)

    def _gather_ok(self) -> bool:
        """A prefill-only step at least as long as the admission window is in flight, no decode
        step is, and the next prefill step would not be full: waiting up to the window for more of
        the burst costs the GPU nothing."""
        eng = self.engine
        pf = eng._pf_inflight
        # (on the CPU a launched step has already run: there is nothing to hide the wait behind)
        if pf is None or eng._inflight is not None or eng.cfg.admit_window_ms <= 0 or eng.device.type != "cuda":
            return False
        cap = eng.cfg.max_prefill_tokens
        s = eng.sched
        # the wait must be hidden: the in-flight step's estimated GPU time covers the admission
        # window (before a prefill rate is measured: a nearly full step)
        toks, tps = sum(pf[0].chunks), self._prefill_tps
        hidden = toks * 1e3 / tps >= eng.cfg.admit_window_ms if tps else toks >= 0.9 * cap
        # prefill_backlog: queued prompts that fit the free slots plus the unprefilled rest of
        # running ones (a chunked prompt's remainder already fills the next step)
        return hidden and len(s.running) < s.cfg.max_num_seqs and s.prefill_backlog() < cap

    def _push_streams(self) -> None:
        for sid, st in list(self._streams.items()):
            seq, sent, cb = st
            out = seq.output_ids
            n = len(out)
            while n > sent and out[n - 1] < 0:  # pipelined decode: placeholders until read back
                n -= 1
            if any(t < 0 for t in out[sent:n]):
                n = sent + next(i for i, t in enumerate(out[sent:n]) if t < 0)
            if n > sent:
                st[1] = n
                try:
                    cb(list(seq.output_ids[sent:n]))
                except Exception:  # noqa: BLE001 - a broken consumer must not stop the engine
                    pass
            if seq.status in (SeqStatus.FINISHED, SeqStatus.ABORTED):
                del self._streams[sid]

    def _step_once(self) -> None:
        eng = self.engine
        if not self._cancels.empty():
            self._apply_cancels()
        self._drain(block=not eng.has_work(), gather=self._gather_ok())
        self._step_cache.clear()
        while eng.step_samples:  # GPU-event step times (back-to-back decode steps)
            self.tpot.record(*eng.step_samples.popleft())
            self._gpu_tpot = True
        if eng.sched.waiting:
            self._expire_waiting()
        self._waiting_est = self._waiting_tokens()
        if not eng.has_work():
            return
        p0, t0 = eng.counters["prefill_steps"], time.perf_counter()
        d0 = eng.counters["decode_steps"]
        paced = eng._inflight is not None or not eng.cfg.pipeline  # this step waits for a GPU step
        ptok0 = eng.runner.n_steps.get("prefill_tokens", 0)
        self._step_t0 = time.monotonic()
        try:
            finished = eng.step()
        finally:
            self._step_t0 = None
        if (paced and not self._gpu_tpot and eng.counters["decode_steps"] > d0
                and eng.counters["prefill_steps"] == p0):
            # (CPU / until event samples arrive) decode-only step: with pipelining, launching
            # step N waits for step N-1, so the interval is one GPU step at (about) this batch size
            rows = eng._inflight[0] if eng._inflight is not None else eng.sched.running
            self.tpot.record(len(rows), (time.perf_counter() - t0) * 1e3, sum(q.num_tokens for q in rows))
        if eng.counters["prefill_steps"] > p0:
            dt = time.perf_counter() - t0
            n = eng.runner.n_steps.get("prefill_tokens", 0) - ptok0
            if n > 0 and dt > 0:
                r = n / dt
                self._prefill_tps = r if self._prefill_tps is None else 0.8 * self._prefill_tps + 0.2 * r
        if self._streams:
            self._push_streams()
        for seq in finished:
            if not seq.params.ignore_eos and seq.finish_reason in ("stop", "length"):
                self.answer_lens.record(sum(1 for t in seq.output_ids if t >= 0))
            fut = seq.user
            if isinstance(fut, Future) and not fut.done():
                self.latencies_ms.append(seq.timings()["latency_ms"])
                fut.set_result((eng.decode_text(seq), seq))
        if finished and eng.trace is not None:
            eng.trace.append((time.perf_counter(), "resolved", len(finished), 0))

    def _on_failure(self, e: BaseException) -> None:
        """A step raised: fail the requests in flight, reset the batch, maybe go unhealthy."""
        eng = self.engine
        eng.counters["step_failures"] += 1
        import logging

        logging.getLogger("engine").error("engine step failed: %r", e, exc_info=e)
        err = RuntimeError(f"engine step failed: {e!r}")
        for s in eng.reset():
            if isinstance(s.user, Future) and not s.user.done():
                s.user.set_exception(err)
        self._streams.clear()
        now = time.monotonic()
        self._failures.append(now)
        while self._failures and now - self._failures[0] > self.failure_window_s:
            self._failures.popleft()
        if len(self._failures) >= self.max_failures or eng.ps.tp_size > 1:
            self._error = e

    def _loop(self) -> None:
        while not self._stop.is_set() and self._error is None:
            try:
                self._step_once()
            except Exception as e:  # noqa: BLE001 - one bad step must not end serving
                self._on_failure(e)
        if self._error is not None:  # unhealthy: refuse what is still queued
            while True:
                try:
                    item = self._q.get_nowait()
                except queue.Empty:
                    break
                if not item[3].done():
                    item[3].set_exception(EngineUnavailable(f"engine unhealthy: {self._error!r}"))

    def stats(self) -> dict:
        d = self.engine.stats()
        lat = sorted(self.latencies_ms)
        if lat:
            d["p50_latency_ms"] = lat[len(lat) // 2]
            d["p99_latency_ms"] = lat[min(len(lat) - 1, int(len(lat) * 0.99))]
        d["queue_depth"] = self._q.qsize()
        d["max_queue"] = self.max_queue
        d["cancelled"] = self.cancelled
        d["rejected"] = self.rejected
        d["expired"] = self.expired
        d["infeasible_rejected"] = self.infeasible
        d["tpot_model_ms"] = self.tpot.snapshot()
        d["prefill_tokens_per_s_est"] = round(self._prefill_tps, 1) if self._prefill_tps else None
        d["healthy"] = self.healthy
        if self._error is not None:
            d["error"] = repr(self._error)
        return d

    def close(self) -> None:
        self._stop.set()
        self._wd_stop.set()
        if self.peer_monitor is not None:
            self.peer_monitor.stop()
        self._thread.join(timeout=10)
        if self._error is None or not self.engine.ps.is_tp:
            self.engine.stop_workers()
