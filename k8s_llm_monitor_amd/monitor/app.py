"""Process assembly for the ``server`` binary (``cmd/server/main.go:23-172``):
config -> cluster client (development-mode fallback) -> metrics manager -> LLM engine ->
analysis service -> REST app.

Cluster backend selection (``k8s.backend``, new): ``kube`` (REST client: kubeconfig or in-cluster
service account), ``fake`` (the deterministic FakeCluster), ``none`` (development mode), ``auto``
(kube if a kubeconfig / in-cluster token exists, else development mode - the reference's
behaviour when it cannot reach a cluster, main.go:43-51).
"""
from __future__ import annotations

import json
import logging
import os
import threading
import time
from dataclasses import dataclass
from typing import Optional

from .config import Config

log = logging.getLogger("server")


@dataclass
class Monitor:
    cfg: Config
    backend: object = None
    client: object = None
    manager: object = None
    engine: object = None
    engine_service: object = None
    analysis: object = None
    app: object = None
    fake: object = None

    def close(self) -> None:
        if self.manager is not None and self.manager.running:
            self.manager.stop()
        if self.engine_service is not None:
            self.engine_service.close()


def make_backend(cfg: Config, fake_seed: int = 0):
    kind = (cfg.k8s.backend or "auto").lower()
    if kind == "none":
        return None
    if kind == "fake":
        from .cluster.fake import FakeCluster

        n = int(os.environ.get("FAKE_CLUSTER_NODES", "3"))
        p = int(os.environ.get("FAKE_CLUSTER_PODS_PER_NODE", "4"))
        return FakeCluster.build(seed=fake_seed, n_nodes=n, pods_per_node=p)
    from .cluster.kube import KubeRESTBackend, KubeConfigError

    try:
        return KubeRESTBackend.from_config(cfg.k8s.kubeconfig)
    except KubeConfigError as e:
        if kind == "kube":
            raise
        log.warning("Failed to create k8s client: %s", e)
        return None


def engine_config(cfg: Config):
    """The in-process engine's EngineConfig from the ``llm:`` block."""
    from ..engine import EngineConfig

    return EngineConfig(model=cfg.llm.model, max_num_seqs=cfg.llm.max_batch, max_model_len=cfg.llm.max_model_len,
                        kv_cache_gb=cfg.llm.kv_cache_gb, use_graphs=cfg.llm.use_graphs, seed=cfg.llm.seed,
                        tp_size=cfg.llm.tp_size, dtype=torch_dtype_name(cfg.llm.dtype),
                        max_prefill_tokens=cfg.llm.max_prefill_tokens, chunked_prefill=cfg.llm.chunked_prefill,
                        prefix_caching=cfg.llm.prefix_caching, weights=cfg.llm.weights or None)


def make_llm_backend(cfg: Config, pstate=None, device: Optional[str] = None):
    """Returns (backend, engine, engine_service).  ``llm.dp_replicas > 1`` (single process,
    TP = 1): the service is a ReplicaRouter over that many engine processes, one per GPU
    (engine/dp.py), and ``engine`` is None (the engines live in the replica processes)."""
    from ..llm.service import LocalEngineBackend, OpenAIBackend, RuleBackend

    prov = (cfg.llm.provider or "").lower()
    if prov in ("local-rocm", "local", "rocm"):
        from ..engine import EngineService, LLMEngine

        ecfg = engine_config(cfg)
        if cfg.llm.dp_replicas > 1 and pstate is None:
            from ..engine.dp import ReplicaRouter, replica_devices

            eng, svc = None, ReplicaRouter(ecfg, replica_devices(cfg.llm.dp_replicas))
        else:
            eng = LLMEngine(ecfg, device=device, pstate=pstate)
            eng.warmup()
            svc = EngineService(eng)
        return (LocalEngineBackend(svc, cfg.llm.max_tokens, cfg.llm.temperature, cfg.llm.top_p, cfg.llm.top_k,
                                   timeout_s=float(cfg.llm.timeout)), eng, svc)
    if prov == "openai":
        return OpenAIBackend(cfg.llm.api_key, cfg.llm.base_url, cfg.llm.model, cfg.llm.max_tokens,
                             cfg.llm.temperature, float(cfg.llm.timeout)), None, None
    return RuleBackend(), None, None


def make_routes(cfg: Config) -> dict:
    """``llm.routes``: analysis type -> an OpenAIBackend on that deployment's OpenAI-compatible
    endpoint (this server's own ``/v1/chat/completions`` when the upstream runs this framework)."""
    from ..llm.service import OpenAIBackend

    return {kind: OpenAIBackend(cfg.llm.api_key or "none", url, cfg.llm.model, cfg.llm.max_tokens,
                                cfg.llm.temperature, float(cfg.llm.timeout))
            for kind, url in (cfg.llm.routes or {}).items() if url}


def build_monitor(cfg: Config, backend=None, start_manager: bool = True, llm: bool = True, pstate=None,
                  device: Optional[str] = None) -> Monitor:
    from ..llm.service import AnalysisService, RecordStore, RuleBackend
    from .analysis.network import RTTTester
    from .cluster.client import K8sClient
    from .metrics.manager import ManagerConfig, MetricsManager
    from .server import MonitorApp

    m = Monitor(cfg=cfg)
    log.info("Starting K8s LLM Monitor...")
    log.info("Server: %s:%d", cfg.server.host, cfg.server.port)
    log.info("K8s Namespace: %s", cfg.k8s.namespace)
    log.info("LLM Provider: %s", cfg.llm.provider)
    m.backend = backend if backend is not None else make_backend(cfg)
    if m.backend is not None:
        client = K8sClient(m.backend, cfg.k8s)
        try:
            v = client.test_connection()
            m.client = client
            log.info("Successfully connected to Kubernetes cluster: %s", v)
        except Exception as e:  # noqa: BLE001
            log.warning("Failed to connect to k8s: %s", e)
            log.warning("Running in development mode without K8s connection")
    else:
        log.warning("Running in development mode without K8s connection")
    if m.client is not None and cfg.metrics.enabled:
        mc = ManagerConfig(namespaces=list(cfg.metrics.namespaces) or ["default"],
                           collect_interval_s=float(cfg.metrics.collect_interval or 30),
                           enable_node=cfg.metrics.enable_node, enable_pod=cfg.metrics.enable_pod,
                           enable_network=cfg.metrics.enable_network, enable_custom=cfg.metrics.enable_custom,
                           enable_uav=True, network_max_pairs=5, network_test_timeout_s=10.0)
        m.manager = MetricsManager(m.backend, mc, RTTTester(m.client))
        if start_manager:
            m.manager.start()
            log.info("Metrics collection started (interval: %d seconds)", cfg.metrics.collect_interval)
    if llm:
        backend_llm, m.engine, m.engine_service = make_llm_backend(cfg, pstate=pstate, device=device)
    else:
        backend_llm = RuleBackend()
    analyzer = None
    m.analysis = AnalysisService(backend_llm, manager=m.manager, client=m.client, analyzer=None,
                                 store=RecordStore(cfg.storage.type, cfg.storage.path),
                                 max_context_events=cfg.analysis.max_context_events,
                                 token_budget=cfg.analysis.prompt_token_budget, max_tokens=cfg.llm.max_tokens,
                                 routes=make_routes(cfg))
    m.app = MonitorApp(m.client, m.manager, m.analysis, m.engine_service, llm_timeout_s=float(cfg.llm.timeout))
    if hasattr(backend_llm, "answer_budget_s"):  # the engine stops generations before the write timeout
        backend_llm.answer_budget_s = m.app.answer_budget_s()
    m.analysis.analyzer = m.app.analyzer if analyzer is None else analyzer
    return m


# --------------------------------------------------------------------------- bench helpers

def build_app_for_bench(engine_service, host: str = "127.0.0.1", port: int = 0, write_timeout_s: float = 600.0,
                        llm_timeout_s: float = 600.0):
    """An HTTP server in this process whose /api/v1/query is served by ``engine_service``
    (FakeCluster behind it, metrics collected once).  Returns (server, port).  The default
    timeouts are the bench's (long waves); ``write_timeout_s=15, llm_timeout_s=30`` is the
    production server's (reference cmd/server/main.go:147-148, config.go:141-145)."""
    from ..llm.service import AnalysisService, LocalEngineBackend
    from .cluster.fake import FakeCluster
    from .cluster.client import K8sClient
    from .config import from_dict
    from .metrics.manager import ManagerConfig, MetricsManager
    from .server import MonitorApp, make_server

    cfg = from_dict({"metrics": {"namespaces": ["default", "kube-system"]}})
    fake = FakeCluster.build(seed=0)
    client = K8sClient(fake, cfg.k8s)
    mgr = MetricsManager(fake, ManagerConfig(namespaces=["default", "kube-system"]))
    mgr.collect()
    backend = LocalEngineBackend(engine_service, max_tokens=2000, temperature=0.1, timeout_s=llm_timeout_s)
    analysis = AnalysisService(backend, manager=mgr, client=client)
    app = MonitorApp(client, mgr, analysis, engine_service, write_timeout_s=write_timeout_s,
                     llm_timeout_s=llm_timeout_s)
    backend.answer_budget_s = app.answer_budget_s()
    analysis.analyzer = app.analyzer
    srv = make_server(app, host, port)
    threading.Thread(target=srv.serve_forever, name="bench-http", daemon=True).start()
    return srv, srv.server_address[1]


class QueryClient:
    """Concurrent /api/v1/query client with persistent state across waves: one worker thread per
    concurrent request, each keeping its HTTP/1.1 keep-alive connection to the server (the REST
    server speaks HTTP/1.1), so a benchmark wave costs no thread spawns and no TCP handshakes on
    either side - as long-lived clients behave."""

    def __init__(self, host: str = "127.0.0.1", workers: int = 64):
        import concurrent.futures as cf
        import threading

        self.host = host
        self.ex = cf.ThreadPoolExecutor(max_workers=workers, thread_name_prefix="client")
        self.workers = workers
        self._tls = threading.local()

    def _conn(self, port: int, fresh: bool = False):
        import http.client
        import socket

        c = getattr(self._tls, "conn", None)
        if fresh or c is None or getattr(self._tls, "port", None) != port:
            if c is not None:
                c.close()
            c = http.client.HTTPConnection(self.host, port, timeout=900)
            c.connect()
            c.sock.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)  # no Nagle wait on keep-alive
            self._tls.conn, self._tls.port = c, port
        return c

    def _request(self, port: int, path: str, body: bytes):
        import http.client

        for attempt in range(2):  # a keep-alive connection the server closed meanwhile: reconnect once
            conn = self._conn(port, fresh=attempt > 0)
            try:
                conn.request("POST", path, body, {"Content-Type": "application/json"})
                r = conn.getresponse()
                data = r.read()
                if r.getheader("Connection", "").lower() == "close":
                    conn.close()
                    self._tls.conn = None
                return r.status, data
            except (http.client.RemoteDisconnected, ConnectionResetError, BrokenPipeError,
                    http.client.CannotSendRequest):
                conn.close()
                self._tls.conn = None
                if attempt:
                    raise
        raise RuntimeError("unreachable")

    def post_queries(self, port: int, items: list, max_new_tokens: int, offsets_s: Optional[list] = None,
                     allow_errors: bool = False) -> list:
        t_start = time.perf_counter()

        def one(i):
            q, ctx = items[i]
            if offsets_s is not None:
                delay = t_start + offsets_s[i] - time.perf_counter()
                if delay > 0:
                    time.sleep(delay)
            body = json.dumps({"question": q, "max_tokens": max_new_tokens, "ignore_eos": True,
                               "context": {"cluster_state": ctx}}).encode()
            t0 = time.perf_counter()
            status, raw = self._request(port, "/api/v1/query", body)
            data = json.loads(raw)
            lat = (time.perf_counter() - t0) * 1e3
            if status != 200 or data.get("status") != "success":
                if allow_errors:
                    return {"http_status": status, "error": data.get("error"), "http_latency_ms": lat,
                            "t_send_s": t0 - t_start}
                raise RuntimeError(f"query failed: HTTP {status}: {data}")
            res = data["result"]
            res["http_status"] = status
            res["http_latency_ms"] = lat
            res["t_send_s"] = t0 - t_start
            return res

        if len(items) > self.workers:
            raise ValueError(f"{len(items)} concurrent requests > {self.workers} client workers")
        return list(self.ex.map(one, range(len(items))))

    def close(self) -> None:
        self.ex.shutdown(wait=True)


_CLIENTS: dict = {}


def post_queries(port: int, items: list, max_new_tokens: int, host: str = "127.0.0.1",
                 concurrency: Optional[int] = None, offsets_s: Optional[list] = None,
                 allow_errors: bool = False) -> list:
    """Fire ``items`` = [(question, context_text)] as concurrent POST /api/v1/query; returns the
    per-request result dicts (answer, timings, ``http_latency_ms``).  ``offsets_s``: open-loop
    arrivals - request i is sent ``offsets_s[i]`` seconds after the call starts (``t_send_s``
    records when it went out).  ``allow_errors``: a non-200 answer becomes
    ``{"http_status": code, "error": ...}`` instead of raising (overload / admission studies).
    Calls with the same (host, concurrency) share one persistent :class:`QueryClient`."""
    n = concurrency or len(items)
    key = (host, n)
    cl = _CLIENTS.get(key)
    if cl is None:
        cl = _CLIENTS[key] = QueryClient(host, n)
    return cl.post_queries(port, items, max_new_tokens, offsets_s=offsets_s, allow_errors=allow_errors)


def post_pod_communication(port: int, pairs: list, max_new_tokens: int, host: str = "127.0.0.1") -> list:
    """Fire ``pairs`` = [(pod_a, pod_b)] as concurrent POST /api/v1/analyze/pod-communication with
    the LLM explanation (BASELINE config 3: the KV-cache + scheduler path); returns per-request
    dicts with the explanation's token counts and the HTTP latency."""
    import concurrent.futures as cf
    import http.client

    def one(pair):
        body = json.dumps({"pod_a": pair[0], "pod_b": pair[1], "max_tokens": max_new_tokens,
                           "ignore_eos": True}).encode()
        conn = http.client.HTTPConnection(host, port, timeout=900)
        t0 = time.perf_counter()
        conn.request("POST", "/api/v1/analyze/pod-communication", body, {"Content-Type": "application/json"})
        r = conn.getresponse()
        data = json.loads(r.read())
        conn.close()
        llm = data.get("llm") or {}
        if r.status != 200 or llm.get("status") != "success":
            raise RuntimeError(f"pod-communication failed: HTTP {r.status}: {data}")
        res = dict(llm["result"])
        res.pop("analysis", None)
        res["http_latency_ms"] = (time.perf_counter() - t0) * 1e3
        return res

    with cf.ThreadPoolExecutor(max_workers=len(pairs)) as ex:
        return list(ex.map(one, pairs))


def bench_pod_pairs(n: int, seed: int = 0) -> list:
    """n (pod_a, pod_b) pairs of the bench FakeCluster (build_app_for_bench uses seed 0)."""
    from .cluster.backend import PODS
    from .cluster.fake import FakeCluster

    fake = FakeCluster.build(seed=seed)
    pods = [f"{p['metadata']['namespace']}/{p['metadata']['name']}" for p in fake.list(PODS, "default")]
    return [(pods[i % len(pods)], pods[(i * 7 + 3) % len(pods)]) for i in range(n)]


def torch_dtype_name(s: str) -> str:
    """``llm.dtype`` ("bf16" / "bfloat16" / "fp16" / "fp32" ...) -> torch dtype attribute name."""
    m = {"bf16": "bfloat16", "bfloat16": "bfloat16", "fp16": "float16", "float16": "float16", "half": "float16",
         "fp32": "float32", "float32": "float32", "float": "float32"}
    try:
        return m[(s or "bf16").lower()]
    except KeyError:
        raise ValueError(f"unsupported llm.dtype {s!r}") from None

