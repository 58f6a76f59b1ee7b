"""REST API server (``cmd/server/main.go``, B1; contract SURVEY.md Appendix A1.1).

All 15 reference routes with their status codes, error strings and Go-``encoding/json`` bodies,
plus the analysis routes the reference only advertised or planned:

  POST /api/v1/query                       {"question", ["max_tokens"], ["stream"]} -> AnalysisResponse
                                           ("stream": true -> text/event-stream: {"delta"} events,
                                           then event "done" carrying the AnalysisResponse)
  POST /api/v1/analyze                     AnalysisRequest {"type", "parameters", "context"}
  GET  /api/v1/analysis[/<request_id>]     stored AnalysisResponse records
  GET  /api/v1/metrics/engine              engine queue / batch / KV-cache / latency stats
  POST /api/v1/analyze/pod-communication   + "llm" key (explanation) when a model is configured
                                           (send "explain": false for the reference body only)

Routing reproduces Go's ServeMux (exact patterns, ``/x/`` subtree patterns, ``/`` fallback to the
static web UI), ``http.Error`` (text/plain, trailing newline, nosniff) and the 405s.  A request
thread that would exceed ``write_timeout_s`` (the reference's 15 s WriteTimeout, main.go:144-149)
answers 504 instead of being cut off silently.
"""
from __future__ import annotations

import json
import socket
import logging
import mimetypes
import os
import signal
import threading
import time
import uuid
from concurrent.futures import TimeoutError as FutTimeout
from http.server import BaseHTTPRequestHandler, ThreadingHTTPServer
from typing import Optional
from urllib.parse import parse_qs, urlparse

from ..utils import gojson
from ..utils.gojson import utcnow
from .types import AnalysisRequest, AnalysisResponse, UAVReport


def _busy_types() -> tuple:
    try:
        from ..engine.engine import EngineOverloaded, EngineUnavailable

        return (EngineOverloaded, EngineUnavailable)
    except Exception:  # noqa: BLE001 - no torch: nothing can be busy
        return (type("_NeverRaised", (Exception,), {}),)


_BUSY = _busy_types()

log = logging.getLogger("server")
WEB_DIR = os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))), "web")
VERSION = "1.0.0"


_POOL = None
_POOL_LOCK = threading.Lock()


def _bounded_pool():
    global _POOL
    if _POOL is None:
        with _POOL_LOCK:
            if _POOL is None:
                import concurrent.futures as cf

                _POOL = cf.ThreadPoolExecutor(max_workers=512, thread_name_prefix="bounded")
    return _POOL


class Reply(Exception):
    def __init__(self, code: int, body: bytes, ctype: str, headers: Optional[dict] = None):
        self.code, self.body, self.ctype, self.headers = code, body, ctype, headers or {}


class StreamReply(Reply):
    """A reply whose body is produced incrementally (``chunks``: an iterator of bytes), written with
    HTTP/1.1 chunked transfer encoding - the Server-Sent Events stream of ``"stream": true``."""

    def __init__(self, code: int, chunks, ctype: str = "text/event-stream", headers: Optional[dict] = None):
        super().__init__(code, b"", ctype, headers)
        self.chunks = chunks

    def collect(self) -> bytes:
        """The whole stream (transport-free callers and tests)."""
        return b"".join(self.chunks)


def sse_event(data, event: Optional[str] = None) -> bytes:
    body = data if isinstance(data, (bytes, bytearray)) else gojson.encode(data).rstrip(b"\n")
    return (b"event: " + event.encode() + b"\n" if event else b"") + b"data: " + bytes(body) + b"\n\n"


def http_error(code: int, msg: str) -> Reply:
    return Reply(code, (msg + "\n").encode(), "text/plain; charset=utf-8", {"X-Content-Type-Options": "nosniff"})


def json_reply(obj, code: int = 200, cors: bool = False) -> Reply:
    return Reply(code, gojson.encode(obj), "application/json", {"Access-Control-Allow-Origin": "*"} if cors else None)


class MonitorApp:
    """The route table; transport-independent (``handle`` is called by the HTTP handler and by tests)."""

    def __init__(self, client=None, manager=None, analysis=None, engine_service=None, web_dir: str = WEB_DIR,
                 write_timeout_s: float = 15.0, llm_timeout_s: float = 30.0):
        self.client = client
        self.manager = manager
        self.analysis = analysis
        self.engine_service = engine_service
        self.web_dir = web_dir
        self.write_timeout_s = write_timeout_s
        self.llm_timeout_s = llm_timeout_s
        self.analyzer = None
        if client is not None:
            from .analysis.network import NetworkAnalyzer

            self.analyzer = NetworkAnalyzer(client)
        self.requests = 0

    # ------------------------------------------------------------------ dispatch (ServeMux)
    def handle(self, method: str, raw_path: str, body: bytes = b"") -> Reply:
        self.requests += 1
        u = urlparse(raw_path)
        path = u.path or "/"
        clean = _clean_path(path)
        if clean != path:  # ServeMux redirects to the canonical path
            loc = clean + (("?" + u.query) if u.query else "")
            return Reply(301, f'<a href="{loc}">Moved Permanently</a>.\n\n'.encode(), "text/html; charset=utf-8",
                         {"Location": loc})
        q = parse_qs(u.query)
        try:
            exact = {
                "/health": self.health,
                "/api/v1/cluster/status": self.cluster_status,
                "/api/v1/pods": self.pods,
                "/api/v1/analyze/pod-communication": self.pod_communication,
                "/api/v1/metrics/cluster": self.metrics_cluster,
                "/api/v1/metrics/nodes": self.metrics_nodes,
                "/api/v1/metrics/pods": self.metrics_pods,
                "/api/v1/metrics/snapshot": self.metrics_snapshot,
                "/api/v1/metrics/network": self.metrics_network,
                "/api/v1/metrics/uav": self.metrics_uav,
                "/api/v1/uav/report": self.uav_report,
                "/api/v1/crd/uav": self.crd_uav,
                "/api/v1/query": self.query,
                "/api/v1/analyze": self.analyze,
                "/api/v1/analysis": self.analysis_list,
                "/api/v1/metrics/engine": self.metrics_engine,
                "/v1/chat/completions": self.chat_completions,
                "/metrics": self.prometheus,
            }
            fn = exact.get(path)
            if fn is not None:
                return fn(method, body, q)
            for prefix, fn in (("/api/v1/metrics/nodes/", self.metrics_node),
                               ("/api/v1/metrics/uav/", self.metrics_uav_node),
                               ("/api/v1/analysis/", self.analysis_get)):
                if path.startswith(prefix):
                    return fn(method, path[len(prefix):])
            return self.static(method, path)
        except Reply as r:
            return r

    # ------------------------------------------------------------------ reference routes
    def health(self, method, body, q) -> Reply:
        """Reference contract (always healthy), except that a configured in-process engine which
        has gone unhealthy (EngineService: repeated step failures / dead engine thread) answers 503
        so a Kubernetes liveness probe restarts the pod."""
        svc = self.engine_service
        if svc is not None and not getattr(svc, "healthy", True):
            return json_reply({"status": "unhealthy", "error": "LLM engine failed", "timestamp": utcnow(),
                               "version": VERSION}, 503)
        return json_reply({"status": "healthy", "timestamp": utcnow(), "version": VERSION})

    def cluster_status(self, method, body, q) -> Reply:
        _only(method, "GET")
        if self.client is None:
            return json_reply({"status": "warning", "message": "K8s client not available - running in development mode",
                               "timestamp": utcnow()})
        try:
            info = self.client.get_cluster_info()
        except Exception as e:  # noqa: BLE001
            raise http_error(500, f"Failed to get cluster info: {e}")
        return json_reply({"status": "success", "cluster_info": info, "timestamp": utcnow()})

    def pods(self, method, body, q) -> Reply:
        _only(method, "GET")
        if self.client is None:
            return json_reply({"status": "warning", "message": "K8s client not available - running in development mode",
                               "pods": [], "timestamp": utcnow()})
        allp = []
        for ns in self.client.namespaces:
            try:
                allp += self.client.get_pods(ns) or []
            except Exception as e:  # noqa: BLE001
                log.warning("Failed to get pods from namespace %s: %s", ns, e)
        return json_reply({"status": "success", "pods": allp, "count": len(allp), "timestamp": utcnow()})

    def pod_communication(self, method, body, q) -> Reply:
        _only(method, "POST")
        if self.client is None:
            raise http_error(503, "K8s client not available - running in development mode")
        req = _decode_object(body)
        if req is None:
            raise http_error(400, "Invalid JSON body")
        a, b = req.get("pod_a"), req.get("pod_b")
        if not isinstance(a, str) or not isinstance(b, str):
            if (a is not None and not isinstance(a, str)) or (b is not None and not isinstance(b, str)):
                raise http_error(400, "Invalid JSON body")
        if not a or not b:
            raise http_error(400, "pod_a and pod_b are required")
        try:
            analysis = self.analyzer.analyze_pod_communication(a, b)
        except Exception as e:  # noqa: BLE001
            raise http_error(500, f"Analysis failed: {e}")
        resp = {"status": "success", "analysis": analysis, "timestamp": utcnow()}
        if self._llm_enabled() and req.get("explain", True) is not False:
            try:
                mt = req.get("max_tokens")  # extension keys (ignored by the reference's decoder)
                mt = int(mt) if isinstance(mt, (int, float)) and not isinstance(mt, bool) and mt > 0 else None
                ie = bool(req.get("ignore_eos", False))
                rec = self._bounded(lambda: self.analysis.explain_pod_communication(analysis, max_tokens=mt,
                                                                                  ignore_eos=ie))
                resp["llm"] = rec
            except FutTimeout:
                resp["llm"] = {"status": "error", "error": "llm timeout"}
            except _BUSY as e:
                resp["llm"] = {"status": "error", "error": f"llm overloaded: {e}"}
        return json_reply(resp)

    def _mgr(self):
        if self.manager is None:
            raise http_error(503, "Metrics manager not available")
        return self.manager

    def metrics_cluster(self, method, body, q) -> Reply:
        _only(method, "GET")
        m = self._mgr()
        return json_reply({"status": "success", "data": m.get_cluster_metrics(), "timestamp": utcnow()}, cors=True)

    def metrics_nodes(self, method, body, q) -> Reply:
        _only(method, "GET")
        s = self._mgr().get_latest_snapshot()
        return json_reply({"status": "success", "data": s.node_metrics, "count": len(s.node_metrics or {}),
                           "timestamp": s.timestamp}, cors=True)

    def metrics_node(self, method, name) -> Reply:
        _only(method, "GET")
        m = self._mgr()
        if not name:
            raise http_error(400, "Node name is required")
        try:
            nm = m.get_node_metrics(name)
        except KeyError as e:
            raise http_error(404, f"Node not found: {e.args[0]}")
        return json_reply({"status": "success", "data": nm, "timestamp": utcnow()}, cors=True)

    def metrics_pods(self, method, body, q) -> Reply:
        _only(method, "GET")
        s = self._mgr().get_latest_snapshot()
        return json_reply({"status": "success", "data": s.pod_metrics, "count": len(s.pod_metrics or {}),
                           "timestamp": s.timestamp}, cors=True)

    def metrics_snapshot(self, method, body, q) -> Reply:
        _only(method, "GET")
        return json_reply({"status": "success", "data": self._mgr().get_latest_snapshot()}, cors=True)

    def metrics_network(self, method, body, q) -> Reply:
        _only(method, "GET")
        n = self._mgr().get_network_metrics()
        return json_reply({"status": "success", "data": n, "count": len(n or []), "timestamp": utcnow()}, cors=True)

    def metrics_uav(self, method, body, q) -> Reply:
        _only(method, "GET")
        u = self._mgr().get_uav_metrics()
        return json_reply({"status": "success", "data": u, "count": len(u), "timestamp": utcnow()}, cors=True)

    def metrics_uav_node(self, method, node) -> Reply:
        _only(method, "GET")
        m = self._mgr()
        if not node:
            raise http_error(400, "Node name is required")
        e = m.get_single_uav_metrics(node)
        if e is None:
            raise http_error(404, f"UAV not found on node: {node}")
        return json_reply({"status": "success", "data": e, "timestamp": utcnow()}, cors=True)

    def uav_report(self, method, body, q) -> Reply:
        _only(method, "POST")
        d = _decode_object(body)
        try:
            r = UAVReport.from_dict(d) if d is not None else None
        except (TypeError, ValueError):
            r = None
        if r is None:
            raise http_error(400, "Invalid JSON body")
        if not r.node_name:
            raise http_error(400, "node_name is required")
        r.uav_id = r.uav_id or f"uav-{r.node_name}"
        if r.timestamp is None or r.timestamp == gojson.ZERO_TIME:
            r.timestamp = utcnow()
        r.source = r.source or "agent"
        r.status = r.status or "active"
        if self.manager is not None:
            self.manager.update_uav_report(r)
        crd_status, crd_err = "unavailable", ""
        if self.client is not None:
            try:
                self.client.upsert_uav_metric(r)
                crd_status = "updated"
            except Exception as e:  # noqa: BLE001
                crd_status, crd_err = "error", str(e)
        resp = {"status": "success", "crd_status": crd_status, "timestamp": utcnow(), "node_name": r.node_name,
                "uav_id": r.uav_id, "uav_status": r.status}
        if r.heartbeat_interval_seconds > 0:
            resp["heartbeat_interval_seconds"] = r.heartbeat_interval_seconds
        if crd_err:
            resp["message"] = crd_err
        return json_reply(resp, cors=True)

    def crd_uav(self, method, body, q) -> Reply:
        _only(method, "GET")
        if self.client is None:
            return json_reply({"status": "error", "message": "K8s client not available"}, 503, cors=True)
        ns = (q.get("namespace") or [""])[0].strip()
        if ns.lower() == "all":
            ns = ""
        try:
            data = self.client.list_uav_metrics_crd(ns)
        except Exception as e:  # noqa: BLE001
            return json_reply({"status": "error", "message": f"failed to list UAV metrics CRDs: {e}"}, 500, cors=True)
        return json_reply({"status": "success", "count": len(data), "data": data, "timestamp": utcnow()}, cors=True)

    # ------------------------------------------------------------------ analysis routes (new)
    def _llm_enabled(self) -> bool:
        from ..llm.service import RuleBackend

        return self.analysis is not None and not isinstance(self.analysis.backend, RuleBackend)

    def answer_budget_s(self) -> float:
        """Time an engine generation may take so the answer still beats the write timeout: the
        engine ends the sequence at this deadline (finish_reason "deadline") - a truncated answer
        instead of a 504 (LocalEngineBackend.answer_budget_s)."""
        return max(0.5, min(self.llm_timeout_s, self.write_timeout_s) - 1.25)

    def _bounded(self, fn, kind: Optional[str] = None):
        """Run fn within the write timeout (leave 0.5 s to write the answer).  One shared pool (no
        thread spawned per request).  The engine itself stops at answer_budget_s (0.75 s earlier),
        so this limit is a backstop; the backend cancels the engine request if it ever fires.
        ``kind``: the analysis type - when the backend that answers it bounds its own wait within
        the same limit (``enforces_deadline``: the in-process engine), fn runs in the handler
        thread: no hand-off to a pool thread and back on every request's path."""
        if kind is not None and self.analysis is not None:
            b = self.analysis.routes.get(kind, self.analysis.backend)
            if getattr(b, "enforces_deadline", False):
                return fn()
        limit = max(0.5, min(self.llm_timeout_s, self.write_timeout_s) - 0.5)
        return _bounded_pool().submit(fn).result(timeout=limit)

    @staticmethod
    def _busy_reply(e: Exception) -> Reply:
        return json_reply(AnalysisResponse(request_id="", status="error", error=f"engine busy: {e}",
                                           timestamp=utcnow()), 503)

    def query(self, method, body, q) -> Reply:
        _only(method, "POST")
        if self.analysis is None:
            raise http_error(503, "Analysis engine not available")
        d = _decode_object(body)
        if d is None:
            raise http_error(400, "Invalid JSON body")
        question = d.get("question")
        if not isinstance(question, str) or not question.strip():
            raise http_error(400, "question is required")
        mt = d.get("max_tokens")
        mt = int(mt) if isinstance(mt, (int, float)) and mt > 0 else None
        ctx = d.get("context")
        ctx_text = ctx.get("cluster_state") if isinstance(ctx, dict) else None
        if ctx_text is not None and not isinstance(ctx_text, str):
            raise http_error(400, "context.cluster_state must be a string")
        if d.get("stream") is True:  # Server-Sent Events: {"delta"} events, then event "done" = the record
            gen = self.analysis.query_stream(question, max_tokens=mt, ignore_eos=bool(d.get("ignore_eos", False)),
                                             context_text=ctx_text)

            def events():
                try:
                    for item in gen:
                        if isinstance(item, str):
                            yield sse_event({"delta": item})
                        else:
                            yield sse_event(item, "done")
                finally:
                    gen.close()  # a client that went away cancels the generation

            return StreamReply(200, events(), headers={"Cache-Control": "no-cache"})
        # inline (handler thread, the engine bounds its own wait) only when nothing before the
        # generation can block: the context is supplied or already built for this snapshot - a
        # new snapshot's context lists events over the K8s API, so it runs under the pool's
        # write-timeout backstop instead
        inline = ctx_text is not None or self.analysis.context_ready()
        try:
            resp = self._bounded(lambda: self.analysis.query(question, max_tokens=mt,
                                                             ignore_eos=bool(d.get("ignore_eos", False)),
                                                             context_text=ctx_text),
                                 kind="query" if inline else None)
        except _BUSY as e:
            return self._busy_reply(e)
        except FutTimeout:
            resp = AnalysisResponse(request_id="", status="error", result={"question": question},
                                    error="answer not ready within the server write timeout", timestamp=utcnow())
            return json_reply(resp, 504)
        return json_reply(resp, 200 if resp.status == "success" else 500)

    def chat_completions(self, method, body, q) -> Reply:
        """OpenAI-compatible generation (the wire format of the reference's ``callLLMAPI``,
        ``provider: openai``): another deployment's ``llm.routes`` entry, or a reference server
        whose ``llm.base_url`` points here, gets its answer from this server's backend.  The
        prompt is the caller's: system message(s) then the user / assistant turns, fitted to the
        local model's window (oldest turns dropped first).  Non-streaming: ``stream: true`` and
        ``stop`` sequences are refused with 400 rather than silently ignored; ``top_p`` is
        honoured."""
        _only(method, "POST")
        if self.analysis is None:
            raise http_error(503, "Analysis engine not available")
        d = _decode_object(body)
        msgs = d.get("messages") if d is not None else None
        if not isinstance(msgs, list) or not msgs or not all(
                isinstance(m, dict) and isinstance(m.get("content"), str) for m in msgs):
            raise http_error(400, "messages must be a non-empty list of {role, content}")
        from ..llm import prompt as P

        parts = [m["content"] for m in msgs]
        if msgs[0].get("role") == "system" and msgs[0]["content"] == P.SYSTEM_PREAMBLE:
            parts = parts[1:]  # every backend adds this server's own preamble
        if d.get("stream") is True:
            raise http_error(400, "stream: true is not supported on /v1/chat/completions")
        if d.get("stop"):
            raise http_error(400, "stop sequences are not supported")
        mt = d.get("max_tokens")
        mt = int(mt) if isinstance(mt, (int, float)) and mt > 0 else None
        temp = d.get("temperature")
        temp = float(temp) if isinstance(temp, (int, float)) else None
        top_p = d.get("top_p")
        top_p = float(top_p) if isinstance(top_p, (int, float)) and 0 < top_p <= 1 else None
        backend = self.analysis.backend
        try:
            prompt = self.analysis.fit_chat(parts, mt)
            g = self._bounded(lambda: backend.generate(prompt, max_tokens=mt, temperature=temp, top_p=top_p))
        except _BUSY as e:
            return self._busy_reply(e)
        except FutTimeout:
            raise http_error(504, "answer not ready within the server write timeout")
        except Exception as e:  # noqa: BLE001
            raise http_error(500, f"{type(e).__name__}: {e}")
        pt, ct = g.get("prompt_tokens"), g.get("completion_tokens")
        usage = {"prompt_tokens": pt, "completion_tokens": ct,
                 "total_tokens": (pt or 0) + (ct or 0) if pt is not None or ct is not None else None}
        return json_reply({"id": "chatcmpl-" + uuid.uuid4().hex, "object": "chat.completion",
                           "created": int(time.time()), "model": g.get("model") or d.get("model", ""),
                           "choices": [{"index": 0, "message": {"role": "assistant", "content": g.get("text", "")},
                                        "finish_reason": g.get("finish_reason") or "stop"}],
                           "usage": usage})

    def analyze(self, method, body, q) -> Reply:
        _only(method, "POST")
        if self.analysis is None:
            raise http_error(503, "Analysis engine not available")
        d = _decode_object(body)
        if d is None:
            raise http_error(400, "Invalid JSON body")
        req = AnalysisRequest(type=str(d.get("type") or ""), parameters=d.get("parameters") or {},
                              context=d.get("context") or {})
        try:
            resp = self._bounded(lambda: self.analysis.analyze(req))
        except _BUSY as e:
            return self._busy_reply(e)
        except ValueError as e:
            raise http_error(400, str(e))
        except FutTimeout:
            return json_reply(AnalysisResponse(request_id="", status="error", error="analysis timed out",
                                               timestamp=utcnow()), 504)
        except Exception as e:  # noqa: BLE001
            raise http_error(500, f"Analysis failed: {e}")
        return json_reply(resp, 200 if resp.status == "success" else 500)

    def analysis_list(self, method, body, q) -> Reply:
        _only(method, "GET")
        if self.analysis is None:
            raise http_error(503, "Analysis engine not available")
        limit = int((q.get("limit") or ["50"])[0] or 50)
        recs = self.analysis.store.list(limit)
        return json_reply({"status": "success", "count": len(recs), "data": recs, "timestamp": utcnow()}, cors=True)

    def analysis_get(self, method, rid) -> Reply:
        _only(method, "GET")
        if self.analysis is None:
            raise http_error(503, "Analysis engine not available")
        rec = self.analysis.store.get(rid)
        if rec is None:
            raise http_error(404, f"Analysis not found: {rid}")
        return json_reply({"status": "success", "data": rec, "timestamp": utcnow()}, cors=True)

    def metrics_engine(self, method, body, q) -> Reply:
        _only(method, "GET")
        if self.engine_service is None:
            raise http_error(503, "LLM engine not available")
        return json_reply({"status": "success", "data": self.engine_service.stats(), "timestamp": utcnow()}, cors=True)

    def prometheus(self, method, body, q) -> Reply:
        """Prometheus text exposition (new; the reference only discussed an exporter,
        docs/uav-collection-summary.md:63-86): HTTP, engine and cluster gauges / counters."""
        _only(method, "GET")
        return Reply(200, prometheus_text(self).encode(), "text/plain; version=0.0.4; charset=utf-8")

    # ------------------------------------------------------------------ static files
    def static(self, method, path) -> Reply:
        rel = "index.html" if path == "/" else path.lstrip("/")
        if path == "/index.html":
            return Reply(301, b"", "text/html; charset=utf-8", {"Location": "./"})
        full = os.path.realpath(os.path.join(self.web_dir, rel))
        if not full.startswith(os.path.realpath(self.web_dir)) or not os.path.isfile(full):
            raise http_error(404, "404 page not found")
        with open(full, "rb") as fh:
            data = fh.read()
        ctype = mimetypes.guess_type(full)[0] or "application/octet-stream"
        if ctype.startswith("text/"):
            ctype += "; charset=utf-8"
        return Reply(200, data, ctype)


_ENGINE_COUNTERS = {"requests": "requests admitted", "finished": "requests finished",
                    "prompt_tokens": "prompt tokens admitted", "generated_tokens": "tokens generated",
                    "prefill_steps": "prefill steps run", "decode_steps": "decode steps run",
                    "preemptions": "sequences preempted (recompute)", "cancelled": "requests cancelled"}
_ENGINE_GAUGES = {"waiting": "sequences waiting", "running": "sequences running",
                  "queue_depth": "requests queued before admission", "kv_blocks_total": "KV-cache blocks",
                  "kv_blocks_free": "free KV-cache blocks", "kv_usage": "KV-cache block usage (0-1)",
                  "p50_latency_ms": "p50 request latency (ms, last 4096)",
                  "p99_latency_ms": "p99 request latency (ms, last 4096)", "healthy": "engine thread healthy",
                  "dp_replicas": "engine replicas behind the router"}
_CLUSTER_GAUGES = ("total_nodes", "healthy_nodes", "total_pods", "running_pods", "total_cpu", "used_cpu",
                   "cpu_usage_rate", "total_memory", "used_memory", "memory_usage_rate", "total_gpus",
                   "available_gpus")


def prometheus_text(app: "MonitorApp") -> str:
    out: list = []

    def metric(name: str, kind: str, help_: str, value, labels: str = "") -> None:
        if isinstance(value, bool):
            value = int(value)
        if not isinstance(value, (int, float)):
            return
        out.append(f"# HELP {name} {help_}\n# TYPE {name} {kind}\n{name}{labels} {value}")

    metric("k8sllm_http_requests_total", "counter", "HTTP requests handled", app.requests)
    if app.engine_service is not None:
        try:
            st = app.engine_service.stats()
        except Exception:  # noqa: BLE001 - a sick engine still exports its health
            st = {"healthy": False}
        model = str(st.get("model", "")).replace('"', "")
        lab = f'{{model="{model}"}}' if model else ""
        for k, h in _ENGINE_COUNTERS.items():
            metric(f"k8sllm_engine_{k}_total", "counter", h, st.get(k), lab)
        for k, h in _ENGINE_GAUGES.items():
            metric(f"k8sllm_engine_{k}", "gauge", h, st.get(k), lab)
    if app.manager is not None:
        try:
            cm = app.manager.get_cluster_metrics()
        except Exception:  # noqa: BLE001
            cm = None
        if cm is not None:
            for k in _CLUSTER_GAUGES:
                metric(f"k8sllm_cluster_{k}", "gauge", f"cluster {k.replace('_', ' ')}", getattr(cm, k, None))
            metric("k8sllm_cluster_healthy", "gauge", "cluster health_status == healthy",
                   int(getattr(cm, "health_status", "") == "healthy"))
    return "\n".join(out) + "\n"


def _only(method: str, allowed: str) -> None:
    if method != allowed:
        raise http_error(405, "Method not allowed")


def _decode_object(body: bytes) -> Optional[dict]:
    try:
        d = json.loads(body or b"")
    except (ValueError, UnicodeDecodeError):
        return None
    return d if isinstance(d, dict) else None


def _clean_path(p: str) -> str:
    """path.Clean + trailing-slash preservation, as ServeMux does."""
    import posixpath

    if not p.startswith("/"):
        p = "/" + p
    c = posixpath.normpath(p)
    if c.startswith("//"):
        c = "/" + c.lstrip("/")
    if p.endswith("/") and c != "/":
        c += "/"
    return c


class _Handler(BaseHTTPRequestHandler):
    app: MonitorApp = None  # set by make_server
    protocol_version = "HTTP/1.1"
    server_version = "k8s-llm-monitor-amd"
    sys_version = ""

    def setup(self):
        super().setup()
        # keep-alive connections: without TCP_NODELAY the body write after the header write waits
        # for the client's delayed ACK (Nagle), ~40 ms per response on Linux
        try:
            self.connection.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
        except OSError:
            pass

    def log_message(self, fmt, *args):  # route access logs to logging (logging.level config)
        log.debug("%s - %s", self.address_string(), fmt % args)

    def _serve(self, method: str) -> None:
        n = int(self.headers.get("Content-Length") or 0)
        body = self.rfile.read(n) if n > 0 else b""
        t0 = time.perf_counter()
        try:
            r = self.app.handle(method, self.path, body)
        except Exception as e:  # noqa: BLE001 - never drop a connection on a bug
            log.exception("handler crashed")
            r = http_error(500, f"internal error: {e}")
        self.send_response(r.code)
        self.send_header("Content-Type", r.ctype)
        for k, v in r.headers.items():
            self.send_header(k, v)
        self.send_header("Date", self.date_time_string())
        if isinstance(r, StreamReply):
            self.send_header("Transfer-Encoding", "chunked")
            self.end_headers()
            try:
                for chunk in r.chunks:
                    if chunk:
                        self.wfile.write(b"%x\r\n%s\r\n" % (len(chunk), chunk))
                        self.wfile.flush()
                self.wfile.write(b"0\r\n\r\n")
            except (BrokenPipeError, ConnectionResetError):  # client went away mid-stream
                self.close_connection = True
                r.chunks.close()
            return
        self.send_header("Content-Length", str(len(r.body)))
        self.end_headers()
        if method != "HEAD":
            self.wfile.write(r.body)
        log.debug("%s %s -> %d in %.2f ms", method, self.path, r.code, (time.perf_counter() - t0) * 1e3)

    def do_GET(self):
        self._serve("GET")

    def do_POST(self):
        self._serve("POST")

    def do_PUT(self):
        self._serve("PUT")

    def do_DELETE(self):
        self._serve("DELETE")

    def do_PATCH(self):
        self._serve("PATCH")

    def do_HEAD(self):
        self._serve("HEAD")

    def do_OPTIONS(self):
        self._serve("OPTIONS")


class MonitorHTTPServer(ThreadingHTTPServer):
    daemon_threads = True
    allow_reuse_address = True
    request_queue_size = 1024

    def handle_error(self, request, client_address) -> None:
        """A client that hangs up mid-request (reset / broken pipe: a load generator or a probe
        closing early) is routine for a server and is logged as one line at debug level; anything
        else keeps socketserver's traceback."""
        import sys

        exc = sys.exc_info()[1]
        if isinstance(exc, (ConnectionResetError, BrokenPipeError, ConnectionAbortedError)):
            logging.getLogger("monitor.http").debug("client %s closed the connection: %r", client_address, exc)
            return
        super().handle_error(request, client_address)


def make_server(app: MonitorApp, host: str = "0.0.0.0", port: int = 8080, read_timeout_s: float = 15.0):
    handler = type("BoundHandler", (_Handler,), {"app": app, "timeout": read_timeout_s})
    return MonitorHTTPServer((host, port), handler)


def serve_until_signal(server, on_stop=None, shutdown_timeout_s: float = 30.0) -> None:
    """ListenAndServe + graceful shutdown on SIGINT/SIGTERM (main.go:152-171)."""
    stop = threading.Event()

    def _sig(signum, frame):
        log.info("Shutting down server...")
        stop.set()

    signal.signal(signal.SIGINT, _sig)
    signal.signal(signal.SIGTERM, _sig)
    t = threading.Thread(target=server.serve_forever, name="http", daemon=True)
    t.start()
    log.info("HTTP Server starting on %s:%d", *server.server_address[:2])
    stop.wait()
    server.shutdown()
    t.join(timeout=shutdown_timeout_s)
    if on_stop:
        on_stop()
    log.info("Server exited")
