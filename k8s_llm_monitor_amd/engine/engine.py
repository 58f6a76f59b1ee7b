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

import queue
import threading
import time
import uuid
from concurrent.futures import Future
from dataclasses import dataclass, field
from typing import Optional, Union

import torch

from ..models.config import ModelConfig, get_config
from ..models.llama import CausalLM
from ..parallel.comm import tp_broadcast_object
from ..parallel.state import ParallelState, get_state
from .block_manager import BlockManager
from .runner import ModelRunner, RunnerConfig
from .scheduler import Scheduler, SchedulerConfig
from .sequence import SamplingParams, Sequence, SeqStatus
from .tokenizer import tokenizer_for


@dataclass
class EngineConfig:
    model: str = "llama-3-8b"
    max_num_seqs: int = 64
    max_model_len: int = 8192
    max_prefill_tokens: int = 16384
    kv_cache_gb: float = 32.0
    num_blocks: Optional[int] = None
    use_graphs: bool = True
    seed: int = 0
    tp_size: int = 1
    dtype: str = "bfloat16"  # compute / weight dtype ("float32" for CPU parity tests)
    model_overrides: dict = field(default_factory=dict)


class _View:
    """What the runner needs of a sequence; built on non-leader TP ranks from the broadcast."""

    __slots__ = ("all_ids", "num_tokens", "block_table", "last_token", "params")

    def __init__(self, all_ids, num_tokens, block_table, last_token, params):
        self.all_ids, self.num_tokens, self.block_table = all_ids, num_tokens, block_table
        self.last_token, self.params = last_token, params


class LLMEngine:
    def __init__(self, cfg: EngineConfig, device: Optional[Union[str, torch.device]] = None,
                 pstate: Optional[ParallelState] = None, model_cfg: Optional[ModelConfig] = None):
        self.cfg = cfg
        self.ps = pstate or get_state()
        if device is None:
            device = self.ps.device if self.ps.device.type == "cuda" else (
                "cuda" if torch.cuda.is_available() else "cpu")
        self.device = torch.device(device)
        mc = model_cfg or get_config(cfg.model)
        if cfg.model_overrides:
            mc = mc.replace(**cfg.model_overrides)
        self.model_cfg = mc
        t0 = time.perf_counter()
        self.model = CausalLM(mc, device=self.device, dtype=getattr(torch, cfg.dtype), seed=cfg.seed, pstate=self.ps)
        self.runner = ModelRunner(self.model, RunnerConfig(
            max_num_seqs=cfg.max_num_seqs, max_model_len=cfg.max_model_len, kv_cache_gb=cfg.kv_cache_gb,
            num_blocks=cfg.num_blocks, use_graphs=cfg.use_graphs, seed=cfg.seed))
        self.blocks = BlockManager(self.runner.num_blocks)
        self.sched = Scheduler(SchedulerConfig(max_num_seqs=cfg.max_num_seqs,
                                               max_prefill_tokens=cfg.max_prefill_tokens,
                                               max_model_len=self.runner.max_len), self.blocks)
        self.tokenizer = tokenizer_for(mc)
        self.eos = set(mc.eos_ids)
        self.init_s = time.perf_counter() - t0
        self.counters = {"requests": 0, "finished": 0, "prompt_tokens": 0, "generated_tokens": 0,
                         "prefill_steps": 0, "decode_steps": 0, "preemptions": 0}
        self.is_leader = self.ps.tp_rank == 0

    # ----------------------------------------------------------------- public API
    def warmup(self) -> None:
        """Capture the decode hipGraphs (all buckets)."""
        t0 = time.perf_counter()
        self.runner.capture_graphs()
        self.graph_s = time.perf_counter() - t0

    def add_request(self, prompt: Union[str, list[int]], params: Optional[SamplingParams] = None,
                    request_id: Optional[str] = None, user=None) -> Sequence:
        ids = self.tokenizer.encode(prompt) if isinstance(prompt, str) else list(prompt)
        limit = self.runner.max_len - 1
        if len(ids) > limit - 1:  # keep room for at least one generated token; trim the middle
            keep = limit - 1
            ids = ids[: keep // 2] + ids[len(ids) - (keep - keep // 2):]
        seq = Sequence(prompt_ids=ids, params=params or SamplingParams(),
                       request_id=request_id or uuid.uuid4().hex[:16], user=user)
        self.sched.add(seq)
        self.counters["requests"] += 1
        self.counters["prompt_tokens"] += len(ids)
        return seq

    def has_work(self) -> bool:
        return self.sched.has_work()

    def step(self) -> list[Sequence]:
        plan = self.sched.schedule()
        self.counters["preemptions"] += len(plan.preempted)
        if plan.empty:
            return []
        if self.ps.tp_size > 1:
            tp_broadcast_object(self._pack(plan), ps=self.ps)
        if plan.is_prefill:
            toks = self.runner.prefill(plan.seqs)
            self.counters["prefill_steps"] += 1
        else:
            toks = self.runner.decode(plan.seqs)
            self.counters["decode_steps"] += 1
        now = time.perf_counter()
        done = []
        for seq, tok in zip(plan.seqs, toks):
            seq.output_ids.append(int(tok))
            self.counters["generated_tokens"] += 1
            if seq.t_first_token is None:
                seq.t_first_token = now
            reason = self._stop_reason(seq, int(tok))
            if reason:
                seq.t_finish = now
                self.sched.finish(seq, reason)
                self.counters["finished"] += 1
                done.append(seq)
        return done

    def _stop_reason(self, seq: Sequence, tok: int) -> Optional[str]:
        p = seq.params
        if not p.ignore_eos and (tok in self.eos or tok in p.stop_token_ids):
            return "stop"
        if len(seq.output_ids) >= p.max_tokens:
            return "length"
        if seq.num_tokens >= self.runner.max_len:
            return "length"
        return None

    def abort(self, seq: Sequence) -> None:
        self.sched.abort(seq)

    def generate(self, prompts: list, params: Optional[SamplingParams] = None) -> list[Sequence]:
        seqs = [self.add_request(p, params) for p in prompts]
        while any(s.status not in (SeqStatus.FINISHED, SeqStatus.ABORTED) for s in seqs):
            self.step()
        return seqs

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
        if plan.is_prefill:
            return (True, [(s.all_ids, s.block_table, _params_t(s.params)) for s in plan.seqs])
        return (False, [(s.last_token, s.num_tokens, s.block_table, _params_t(s.params)) for s in plan.seqs])

    def worker_loop(self) -> None:
        """Non-leader TP ranks: mirror the leader's steps until it broadcasts ``None``."""
        while True:
            msg = tp_broadcast_object(None, ps=self.ps)
            if msg is None:
                return
            is_prefill, items = msg
            if is_prefill:
                views = [_View(ids, len(ids), bt, ids[-1], SamplingParams(*p)) for ids, bt, p in items]
                self.runner.prefill(views)
            else:
                views = [_View(None, n, bt, last, SamplingParams(*p)) for last, n, bt, p in items]
                self.runner.decode(views)

    def stop_workers(self) -> None:
        if self.ps.tp_size > 1 and self.is_leader:
            tp_broadcast_object(None, ps=self.ps)


def _params_t(p: SamplingParams) -> tuple:
    return (p.max_tokens, p.temperature, p.top_k, p.top_p, p.ignore_eos, tuple(p.stop_token_ids))


class EngineService:
    """Runs an LLMEngine on its own thread; thread-safe ``submit`` returns a Future that resolves
    to ``(text, sequence)``."""

    def __init__(self, engine: LLMEngine):
        self.engine = engine
        self._q: queue.Queue = queue.Queue()
        self._stop = threading.Event()
        self._thread = threading.Thread(target=self._loop, name="llm-engine", daemon=True)
        self._lock = threading.Lock()
        self._error: Optional[BaseException] = None
        self.latencies_ms: list[float] = []
        self._thread.start()

    def submit(self, prompt: Union[str, list[int]], params: Optional[SamplingParams] = None,
               request_id: Optional[str] = None) -> Future:
        fut: Future = Future()
        if self._error is not None:
            fut.set_exception(RuntimeError(f"engine failed: {self._error!r}"))
            return fut
        self._q.put((prompt, params, request_id, fut))
        return fut

    def _drain(self, block: bool) -> None:
        try:
            item = self._q.get(block=block, timeout=0.05 if block else None)
        except queue.Empty:
            return
        while item is not None:
            prompt, params, rid, fut = item
            try:
                self.engine.add_request(prompt, params, rid, user=fut)
            except Exception as e:  # noqa: BLE001 - reject this request only
                fut.set_exception(e)
            try:
                item = self._q.get_nowait()
            except queue.Empty:
                item = None

    def _loop(self) -> None:
        eng = self.engine
        try:
            while not self._stop.is_set():
                self._drain(block=not eng.has_work())
                if not eng.has_work():
                    continue
                for seq in eng.step():
                    fut = seq.user
                    if isinstance(fut, Future) and not fut.done():
                        self.latencies_ms.append(seq.timings()["latency_ms"])
                        fut.set_result((eng.decode_text(seq), seq))
        except BaseException as e:  # noqa: BLE001 - surface to every waiter
            self._error = e
            for s in list(eng.sched.running) + list(eng.sched.waiting):
                if isinstance(s.user, Future) and not s.user.done():
                    s.user.set_exception(RuntimeError(f"engine failed: {e!r}"))
            raise

    def stats(self) -> dict:
        d = self.engine.stats()
        lat = sorted(self.latencies_ms[-4096:])
        if lat:
            d["p50_latency_ms"] = lat[len(lat) // 2]
            d["p99_latency_ms"] = lat[min(len(lat) - 1, int(len(lat) * 0.99))]
        d["queue_depth"] = self._q.qsize()
        d["healthy"] = self._error is None
        return d

    def close(self) -> None:
        self._stop.set()
        self._thread.join(timeout=10)
        self.engine.stop_workers()
