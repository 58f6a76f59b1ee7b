"""The analysis engine the reference only planned (``internal/llm``, docs/development-guide.md:39-64).

``AnalysisService`` turns questions and ``AnalysisRequest``s (types ``pod_communication`` |
``anomaly_detection`` | ``root_cause``, pkg/models/models.go:86-90) into ``AnalysisResponse``
records (models.go:93-99) using a text-generation backend:

* ``LocalEngineBackend`` - the in-process PyTorch-ROCm engine (``llm.provider: local-rocm``):
  continuous batching across concurrent HTTP requests, hipGraph decode, HIP kernels;
* ``OpenAIBackend``      - the reference's intended remote call (``provider: openai``,
  ``OPENAI_API_KEY``/``OPENAI_BASE_URL``, config.go:141-182), an OpenAI-compatible
  ``/chat/completions`` POST with ``llm.timeout``;
* ``RuleBackend``        - no model: a deterministic summary of the rule findings (dev mode).

Records are kept by ``RecordStore`` (``storage.type: memory`` ring buffer, or ``file`` JSON lines;
the reference's redis/postgres settings are accepted but unsupported offline).
"""
from __future__ import annotations

import json
import logging
import os
import threading
import time
import urllib.request
import uuid
from collections import OrderedDict
from concurrent.futures import TimeoutError as FutTimeout
from typing import Optional

from ..monitor.types import AnalysisRequest, AnalysisResponse
from ..utils import gojson
from ..utils.gojson import utcnow
from . import prompt as P

log = logging.getLogger("llm")


class GenResult(dict):
    """{text, prompt_tokens, completion_tokens, latency_ms, ttft_ms, model, provider}"""


class AnswerBudgetExceeded(FutTimeout):
    """The in-process engine's answer budget ran out (LocalEngineBackend.generate): the HTTP layer
    answers 504.  Its own type, so that other timeouts (a routed backend's socket timeout, which
    IS ``concurrent.futures.TimeoutError`` on Python >= 3.11) still become error records."""


class LocalEngineBackend:
    provider = "local-rocm"
    # generate() never waits past answer_budget_s + 0.75 s (the engine ends the sequence at the
    # budget): the HTTP layer's write-timeout backstop is already enforced here
    enforces_deadline = True

    def __init__(self, service, max_tokens: int = 2000, temperature: float = 0.1, top_p: float = 1.0,
                 top_k: int = 0, timeout_s: float = 30.0, answer_budget_s: Optional[float] = None):
        """``timeout_s`` is ``llm.timeout``.  ``answer_budget_s`` (default: timeout_s): the time a
        synchronous answer may take - the server sets it below its write timeout
        (``answer_budget``) so the engine ends the generation at the deadline with
        finish_reason "deadline" and the caller gets the answer generated so far, instead of a 504
        while the GPU keeps generating for a client that has gone."""
        from ..engine import SamplingParams

        self.svc = service
        self.model = service.engine.model_cfg.name
        self.default = SamplingParams(max_tokens=max_tokens, temperature=temperature, top_p=top_p, top_k=top_k)
        self.timeout_s = timeout_s
        self.answer_budget_s = answer_budget_s if answer_budget_s is not None else (timeout_s if timeout_s > 0 else None)
        self.tokenizer = service.engine.tokenizer
        eng = service.engine
        mml = getattr(getattr(eng, "cfg", None), "max_model_len", None) or (1 << 30)
        self.max_len = min(int(mml), int(eng.model_cfg.max_position))  # the engine's per-sequence cap

    def max_prompt_tokens(self, max_tokens: Optional[int] = None) -> int:
        """Prompt tokens that still leave room for ``max_tokens`` answer tokens (preamble included);
        the answer's reservation is capped at half the window (llm.max_tokens 2000 against a
        1024-token GPT-2 would otherwise leave no room for the cluster context)."""
        return self.max_len - 1 - min(max_tokens or self.default.max_tokens, self.max_len // 2)

    def count_tokens(self, text: str) -> int:
        return len(self.tokenizer.encode(text, bos=False))

    def generate(self, prompt: str, max_tokens: Optional[int] = None, temperature: Optional[float] = None,
                 request_id: Optional[str] = None, ignore_eos: bool = False,
                 top_p: Optional[float] = None) -> GenResult:
        from ..engine import SamplingParams

        d = self.default
        p = SamplingParams(max_tokens=max_tokens or d.max_tokens,
                           temperature=d.temperature if temperature is None else temperature,
                           top_k=d.top_k, top_p=d.top_p if top_p is None else top_p, ignore_eos=ignore_eos)
        budget = self.answer_budget_s
        fut = self.svc.submit(P.SYSTEM_PREAMBLE + prompt, p, request_id,
                              deadline=time.perf_counter() + budget if budget else None)
        try:
            # the engine stops the sequence at the deadline; the grace covers the last step + detokenize
            # (budget + 0.75 s = the server's write timeout - 0.5 s: the HTTP layer's backstop limit)
            text, seq = fut.result(timeout=budget + 0.75 if budget else None)
        except FutTimeout:
            self.svc.cancel(fut)  # free the KV blocks: nobody waits for this answer any more
            # a futures TimeoutError: the HTTP layer answers it 504, as its own write-timeout backstop
            raise AnswerBudgetExceeded("answer not ready within the answer budget") from None
        t = seq.timings()
        return GenResult(text=text, model=self.model, provider=self.provider, finish_reason=seq.finish_reason, **t)


    def stream(self, prompt: str, max_tokens: Optional[int] = None, temperature: Optional[float] = None,
               request_id: Optional[str] = None, ignore_eos: bool = False):
        """Generator: text deltas (str) as the engine produces tokens, then the final GenResult.
        The engine thread only enqueues token ids; detokenization runs here, incrementally (a
        sliding window, so the cost per token does not grow with the answer)."""
        import queue

        from ..engine import SamplingParams

        d = self.default
        p = SamplingParams(max_tokens=max_tokens or d.max_tokens,
                           temperature=d.temperature if temperature is None else temperature,
                           top_k=d.top_k, top_p=d.top_p, ignore_eos=ignore_eos)
        q: queue.SimpleQueue = queue.SimpleQueue()
        fut = self.svc.submit(P.SYSTEM_PREAMBLE + prompt, p, request_id, on_tokens=q.put,
                              deadline=time.perf_counter() + self.timeout_s if self.timeout_s > 0 else None)
        det = IncrementalDetokenizer(self.tokenizer)
        deadline = time.monotonic() + self.timeout_s if self.timeout_s > 0 else None
        try:
            while True:
                try:
                    ids = q.get(timeout=0.05)
                except queue.Empty:
                    if fut.done() and q.empty():
                        break
                    if deadline is not None and time.monotonic() > deadline:
                        raise TimeoutError("llm.timeout exceeded while streaming")
                    continue
                delta = det.add(ids)
                if delta:
                    yield delta
        finally:
            if not fut.done() and hasattr(self.svc, "cancel"):  # consumer gone / timed out: free the KV
                self.svc.cancel(fut)
        text, seq = fut.result()
        tail = det.flush()
        if tail:
            yield tail
        yield GenResult(text=text, model=self.model, provider=self.provider, finish_reason=seq.finish_reason,
                        **seq.timings())


class IncrementalDetokenizer:
    """Token ids -> text deltas for streaming: each call re-decodes only the ids since the previous
    emission boundary (prefix / read offsets, so the cost per token does not grow with the answer)
    and holds output back while the text ends inside a multi-byte UTF-8 character (U+FFFD)."""

    def __init__(self, tokenizer):
        self.tok = tokenizer
        self.ids: list[int] = []
        self.prefix = 0  # start of the previously emitted chunk (a character boundary)
        self.read = 0  # ids already emitted as text

    def add(self, ids) -> str:
        self.ids.extend(int(t) for t in ids)
        prev = self.tok.decode(self.ids[self.prefix:self.read])
        cur = self.tok.decode(self.ids[self.prefix:])
        if len(cur) <= len(prev) or cur.endswith("\ufffd"):
            return ""
        self.prefix, self.read = self.read, len(self.ids)
        return cur[len(prev):]

    def flush(self) -> str:
        """Whatever is still held back (the answer ended inside a character)."""
        if self.read == len(self.ids):
            return ""
        prev = self.tok.decode(self.ids[self.prefix:self.read])
        cur = self.tok.decode(self.ids[self.prefix:])
        self.prefix, self.read = self.read, len(self.ids)
        return cur[len(prev):]


class OpenAIBackend:
    provider = "openai"

    def __init__(self, api_key: str, base_url: str, model: str, max_tokens: int, temperature: float, timeout_s: float):
        self.api_key, self.model = api_key, model
        self.base_url = (base_url or "https://api.openai.com/v1").rstrip("/")
        self.max_tokens, self.temperature, self.timeout_s = max_tokens, temperature, timeout_s

    def count_tokens(self, text: str) -> int:
        return max(1, len(text.encode()) // 3)

    def generate(self, prompt: str, max_tokens: Optional[int] = None, temperature: Optional[float] = None,
                 request_id: Optional[str] = None, ignore_eos: bool = False,
                 top_p: Optional[float] = None) -> GenResult:
        if not self.api_key:
            raise RuntimeError("llm.api_key / OPENAI_API_KEY not configured")
        req_d = {"model": self.model, "max_tokens": max_tokens or self.max_tokens,
                 "temperature": self.temperature if temperature is None else temperature,
                 "messages": [{"role": "system", "content": P.SYSTEM_PREAMBLE},
                              {"role": "user", "content": prompt}]}
        if top_p is not None:
            req_d["top_p"] = top_p
        body = json.dumps(req_d).encode()
        req = urllib.request.Request(self.base_url + "/chat/completions", data=body, method="POST",
                                     headers={"Content-Type": "application/json",
                                              "Authorization": f"Bearer {self.api_key}"})
        t0 = time.perf_counter()
        with urllib.request.urlopen(req, timeout=self.timeout_s) as r:
            d = json.loads(r.read())
        usage = d.get("usage") or {}
        return GenResult(text=d["choices"][0]["message"]["content"], model=d.get("model") or self.model,
                         provider=self.provider,
                         prompt_tokens=usage.get("prompt_tokens"), completion_tokens=usage.get("completion_tokens"),
                         latency_ms=round((time.perf_counter() - t0) * 1e3, 3), ttft_ms=None,
                         finish_reason=d["choices"][0].get("finish_reason"))


class RuleBackend:
    provider = "rules"
    model = "rule-engine"

    def count_tokens(self, text: str) -> int:
        return max(1, len(text.encode()) // 3)

    def generate(self, prompt: str, max_tokens: Optional[int] = None, temperature: Optional[float] = None,
                 request_id: Optional[str] = None, ignore_eos: bool = False,
                 top_p: Optional[float] = None) -> GenResult:
        flagged = [ln.strip() for ln in prompt.splitlines()
                   if any(k in ln for k in ("[资源压力]", "[不健康]", "状态=", "接近限制", "不通", "告警", "UAV "))]
        text = ("未发现明显异常。" if not flagged else
                "规则引擎摘要 (未配置本地模型):\n" + "\n".join(flagged[:50]))
        return GenResult(text=text, model=self.model, provider=self.provider, prompt_tokens=self.count_tokens(prompt),
                         completion_tokens=self.count_tokens(text), latency_ms=0.0, ttft_ms=0.0,
                         finish_reason="stop")


class RecordStore:
    """Analysis records by request id (bounded ring buffer; optional JSON-lines persistence so
    records survive a restart - the reference keeps nothing, SURVEY.md §5 checkpoint/resume)."""

    def __init__(self, kind: str = "memory", path: str = "", capacity: int = 10000):
        self.kind, self.capacity = kind, capacity
        self._d: OrderedDict = OrderedDict()
        self._lock = threading.Lock()
        self.path = None
        if kind == "file":
            self.path = os.path.join(path or ".", "analysis_records.jsonl")
            os.makedirs(os.path.dirname(self.path) or ".", exist_ok=True)
            if os.path.exists(self.path):
                with open(self.path, encoding="utf-8") as fh:
                    for line in fh:
                        try:
                            d = json.loads(line)
                            self._d[d["request_id"]] = d
                        except (ValueError, KeyError):
                            continue
        elif kind not in ("memory", ""):
            log.warning("storage.type %r is not available offline; using memory", kind)

    def put(self, resp: AnalysisResponse) -> None:
        """Keep the record as it is (a finished response is never mutated): the Go-encoding round
        trip into plain values happens when a record is read back (``get`` / ``list``, rare), not
        on every answer's path - it cost as much as encoding the HTTP reply itself."""
        line = gojson.dumps(resp) + "\n" if self.path else None
        with self._lock:
            self._d[resp.request_id] = resp
            while len(self._d) > self.capacity:
                self._d.popitem(last=False)
            if line is not None:
                with open(self.path, "a", encoding="utf-8") as fh:
                    fh.write(line)

    @staticmethod
    def _plain(rec):
        return rec if isinstance(rec, dict) else gojson.to_plain(rec)

    def get(self, rid: str) -> Optional[dict]:
        with self._lock:
            rec = self._d.get(rid)
        return None if rec is None else self._plain(rec)

    def list(self, limit: int = 50) -> list:
        with self._lock:
            recs = list(self._d.values())[-limit:]
        return [self._plain(r) for r in recs]

    def __len__(self) -> int:
        return len(self._d)


class AnalysisService:
    def __init__(self, backend, manager=None, client=None, analyzer=None, store: Optional[RecordStore] = None,
                 max_context_events: int = 100, token_budget: int = 6144, max_tokens: Optional[int] = None,
                 routes: Optional[dict] = None):
        """``routes``: analysis type -> backend that answers it (``llm.routes``: the root-cause
        model on a 70B TP=8 deployment, anomaly detection on Mixtral - ``models.go:86-90``); the
        prompt is built here, from this server's cluster context, and only generation is remote."""
        self.backend = backend
        self.routes = dict(routes or {})
        self.manager = manager
        self.client = client
        self.analyzer = analyzer
        self.store = store or RecordStore()
        self.max_events = max_context_events
        self.token_budget = token_budget
        self.max_tokens = max_tokens
        self._ctx_cache: tuple = (None, "")
        self._ctx_lock = threading.Lock()

    # ------------------------------------------------------------------ context
    def _events(self) -> list:
        if self.client is None:
            return []
        out = []
        for ns in self.client.namespaces:
            try:
                out += self.client.get_events(ns, limit=self.max_events) or []
            except Exception as e:  # noqa: BLE001
                log.warning("events for %s unavailable: %s", ns, e)
        out.sort(key=lambda e: e.timestamp or utcnow())
        return out[-self.max_events:]

    def cluster_context(self) -> str:
        if self.manager is None:
            return "\n(集群指标不可用: metrics manager not available)\n"
        snap = self.manager.get_latest_snapshot()
        key = (id(snap), snap.timestamp)
        with self._ctx_lock:
            if self._ctx_cache[0] == key:
                return self._ctx_cache[1]
        ctx = P.build_cluster_context(snap, self._events(), self.manager.get_uav_metrics(), self.max_events)
        ctx = P.trim_to_budget(ctx, lambda s: [0] * self.backend.count_tokens(s), self.token_budget)
        with self._ctx_lock:
            self._ctx_cache = (key, ctx)
        return ctx

    def context_ready(self) -> bool:
        """True when cluster_context() would return without touching the K8s API (no metrics
        manager, or the current snapshot's context is cached)."""
        if self.manager is None:
            return True
        snap = self.manager.get_latest_snapshot()
        with self._ctx_lock:
            return self._ctx_cache[0] == (id(snap), snap.timestamp)

    def backend_for(self, kind: str):
        """The backend that answers analysis type ``kind`` (``llm.routes``, else the default)."""
        return self.routes.get(kind, self.backend)

    def _fit(self, ctx: str, frame: str, max_tokens: Optional[int], kind: str = "query") -> str:
        """Trim the cluster context so that the whole prompt (``frame`` = the prompt without the
        context) plus ``max_tokens`` answer tokens fit the window of the model that answers
        ``kind`` (a routed deployment's, not the local one's), counted with that backend's
        tokenizer: a 1024-token GPT-2 would otherwise get its prompt cut in the middle by the
        engine and room for one answer token.  A backend that publishes no window (a remote
        OpenAI-compatible server) gets the context untrimmed.  Cheap when nothing can overflow: a
        byte-level BPE token covers >= 1 byte, so a prompt of fewer bytes than the budget is never
        tokenized here."""
        backend = self.backend_for(kind)
        limit = getattr(backend, "max_prompt_tokens", None)
        count = getattr(backend, "count_tokens", None)
        if limit is None or count is None:
            return ctx
        budget = limit(max_tokens or self.max_tokens) - len(P.SYSTEM_PREAMBLE.encode())
        if len(ctx.encode()) + len(frame.encode()) <= budget:
            return ctx
        budget -= count(frame) + 8
        return P.trim_to_budget(ctx, lambda t: [0] * count(t), max(budget, 16))

    def fit_chat(self, parts: list, max_tokens: Optional[int]) -> str:
        """The turns of an OpenAI-style chat joined into one prompt that fits the local model's
        window with ``max_tokens`` answer tokens: the oldest turns are dropped first; a last turn
        that alone is too long keeps its head and tail (trim_to_budget)."""
        limit = getattr(self.backend, "max_prompt_tokens", None)
        count = getattr(self.backend, "count_tokens", None)
        joined = "\n\n".join(parts)
        if limit is None or count is None:
            return joined
        budget = limit(max_tokens or self.max_tokens) - len(P.SYSTEM_PREAMBLE.encode())
        if len(joined.encode()) <= budget:
            return joined
        budget = max(budget, 16)
        parts = list(parts)
        while len(parts) > 1 and count("\n\n".join(parts)) > budget:
            parts.pop(0)
        return P.trim_to_budget("\n\n".join(parts), lambda t: [0] * count(t), budget)

    # ------------------------------------------------------------------ entry points
    def _respond(self, rid: str, kind: str, prompt: str, extra: dict, max_tokens: Optional[int] = None,
                 ignore_eos: bool = False) -> AnalysisResponse:
        from ..engine import EngineOverloaded, EngineUnavailable

        backend = self.backend_for(kind)
        try:
            g = backend.generate(prompt, max_tokens=max_tokens or self.max_tokens, request_id=rid,
                                 ignore_eos=ignore_eos)
            result = {"type": kind, "answer": g.pop("text"), **g, **extra}
            resp = AnalysisResponse(request_id=rid, status="success", result=result, timestamp=utcnow())
        except (EngineOverloaded, EngineUnavailable):
            raise  # admission refused: the HTTP layer answers 503 (nothing to record)
        except AnswerBudgetExceeded:
            raise  # the answer budget ran out: the HTTP layer answers 504
        except Exception as e:  # noqa: BLE001 - an engine failure becomes an error record, not a 500
            log.error("analysis %s failed: %s", rid, e)
            resp = AnalysisResponse(request_id=rid, status="error", result={"type": kind, **extra},
                                    error=f"{type(e).__name__}: {e}", timestamp=utcnow())
        self.store.put(resp)
        return resp

    def query_stream(self, question: str, max_tokens: Optional[int] = None, ignore_eos: bool = False,
                     context_text: Optional[str] = None):
        """Streaming form of :meth:`query` (``"stream": true``): yields text deltas, then the stored
        AnalysisResponse.  Backends without token streaming yield the whole answer as one delta."""
        rid = uuid.uuid4().hex
        ctx = context_text if context_text else self.cluster_context()
        mt = max_tokens or self.max_tokens
        ctx = self._fit(ctx, P.build_query_prompt("", question), mt, "query")
        prompt = P.build_query_prompt(ctx, question)
        extra = {"question": question}
        try:
            if hasattr(self.backend, "stream"):
                g = None
                for item in self.backend.stream(prompt, max_tokens=mt, request_id=rid, ignore_eos=ignore_eos):
                    if isinstance(item, str):
                        yield item
                    else:
                        g = item
            else:
                g = self.backend.generate(prompt, max_tokens=mt, request_id=rid, ignore_eos=ignore_eos)
                yield g["text"]
            result = {"type": "query", "answer": g.pop("text"), **g, **extra}
            resp = AnalysisResponse(request_id=rid, status="success", result=result, timestamp=utcnow())
        except Exception as e:  # noqa: BLE001 - an engine failure becomes an error record
            log.error("analysis %s failed: %s", rid, e)
            resp = AnalysisResponse(request_id=rid, status="error", result={"type": "query", **extra},
                                    error=f"{type(e).__name__}: {e}", timestamp=utcnow())
        self.store.put(resp)
        yield resp

    def query(self, question: str, max_tokens: Optional[int] = None, ignore_eos: bool = False,
              context_text: Optional[str] = None) -> AnalysisResponse:
        """POST /api/v1/query (README.md:91-96; not implemented by the reference).  ``context_text``
        lets a caller supply the cluster state itself (e.g. another collector's snapshot)."""
        rid = uuid.uuid4().hex
        ctx = context_text if context_text else self.cluster_context()
        ctx = self._fit(ctx, P.build_query_prompt("", question), max_tokens, "query")
        prompt = P.build_query_prompt(ctx, question)
        return self._respond(rid, "query", prompt, {"question": question}, max_tokens, ignore_eos)

    def analyze(self, req: AnalysisRequest) -> AnalysisResponse:
        kind = req.type or "anomaly_detection"
        params = req.parameters or {}
        if kind == "pod_communication":
            a, b = params.get("pod_a"), params.get("pod_b")
            if not a or not b or self.analyzer is None:
                raise ValueError("pod_a and pod_b are required" if self.analyzer else "K8s client not available")
            analysis = self.analyzer.analyze_pod_communication(a, b)
            return self.explain_pod_communication(analysis)
        if kind not in ("anomaly_detection", "root_cause"):
            raise ValueError(f"unknown analysis type: {kind}")
        mt = int(params.get("max_tokens") or 0) or None
        ctx = self._fit(self.cluster_context(), P.build_analysis_prompt(kind, "", params), mt, kind)
        prompt = P.build_analysis_prompt(kind, ctx, params)
        return self._respond(uuid.uuid4().hex, kind, prompt, {"parameters": params}, mt)

    def explain_pod_communication(self, analysis, max_tokens: Optional[int] = None,
                                  ignore_eos: bool = False) -> AnalysisResponse:
        facts = []
        if self.client is not None:
            from ..monitor.analysis.network import parse_pod_name

            for ref in (analysis.pod_a, analysis.pod_b):
                try:
                    ns, n = parse_pod_name(ref)
                    p = self.client.get_pod(ns, n)
                    facts.append(f"- {ns}/{n}: 状态={p.status}, 节点={p.node_name}, IP={p.ip}, 标签={p.labels or {}}")
                except Exception as e:  # noqa: BLE001
                    facts.append(f"- {ref}: {e}")
        rtt = ""
        last = getattr(self.analyzer, "last_rtt", None)
        if last is not None:
            rtt = (f"RTT测试: 成功率 {last.success_rate:.1f}%, 平均 {last.average_rtt:.2f}ms, "
                   f"评级 {last.latency}\n")
        prompt = P.build_pod_communication_prompt(analysis, "\n".join(facts), rtt)
        return self._respond(uuid.uuid4().hex, "pod_communication", prompt, {"analysis": gojson.to_plain(analysis)},
                             max_tokens, ignore_eos)
