"""REST contract tests: every route, dev mode and FakeCluster."""
import http.client
import json
import time
import os
import threading

import pytest

from k8s_llm_monitor_amd.monitor.app import build_monitor
from k8s_llm_monitor_amd.monitor.cluster.fake import FakeCluster
from k8s_llm_monitor_amd.monitor.config import from_dict
from k8s_llm_monitor_amd.monitor.server import MonitorApp, make_server


def J(r):
    assert r.ctype == "application/json", r.ctype
    assert r.body.endswith(b"\n")
    return json.loads(r.body)


@pytest.fixture()
def mon():
    cfg = from_dict({"k8s": {"watch_namespaces": "default,kube-system"},
                     "metrics": {"namespaces": ["default", "kube-system"], "enable_network": True},
                     "llm": {"provider": "none"}})
    m = build_monitor(cfg, backend=FakeCluster.build(seed=2), start_manager=False, llm=True)
    m.manager.collect()
    return m


def test_dev_mode_contract():
    a = MonitorApp()
    assert J(a.handle("GET", "/health"))["version"] == "1.0.0"
    d = J(a.handle("GET", "/api/v1/cluster/status"))
    assert set(d) == {"message", "status", "timestamp"} and d["status"] == "warning"
    assert d["message"] == "K8s client not available - running in development mode"
    d = J(a.handle("GET", "/api/v1/pods"))
    assert d["pods"] == [] and d["status"] == "warning"
    r = a.handle("POST", "/api/v1/analyze/pod-communication", b"{}")
    assert r.code == 503 and r.body == b"K8s client not available - running in development mode\n"
    for p in ("/api/v1/metrics/cluster", "/api/v1/metrics/nodes", "/api/v1/metrics/nodes/x", "/api/v1/metrics/pods",
              "/api/v1/metrics/snapshot", "/api/v1/metrics/network", "/api/v1/metrics/uav", "/api/v1/metrics/uav/x"):
        r = a.handle("GET", p)
        assert (r.code, r.body, r.ctype) == (503, b"Metrics manager not available\n", "text/plain; charset=utf-8"), p
    r = a.handle("GET", "/api/v1/crd/uav")
    assert r.code == 503 and J(r) == {"message": "K8s client not available", "status": "error"}
    r = a.handle("POST", "/api/v1/uav/report", b'{"node_name":"n1"}')
    d = J(r)
    assert r.code == 200 and d["crd_status"] == "unavailable" and d["uav_id"] == "uav-n1" and d["uav_status"] == "active"
    assert r.headers.get("Access-Control-Allow-Origin") == "*"


def test_methods_and_errors(mon):
    a = mon.app
    for p in ("/api/v1/cluster/status", "/api/v1/pods", "/api/v1/metrics/cluster", "/api/v1/crd/uav"):
        r = a.handle("POST", p)
        assert r.code == 405 and r.body == b"Method not allowed\n"
    assert a.handle("GET", "/api/v1/analyze/pod-communication").code == 405
    assert a.handle("GET", "/api/v1/uav/report").code == 405
    r = a.handle("POST", "/api/v1/analyze/pod-communication", b"{bad")
    assert (r.code, r.body) == (400, b"Invalid JSON body\n")
    r = a.handle("POST", "/api/v1/analyze/pod-communication", b'{"pod_a":"x"}')
    assert (r.code, r.body) == (400, b"pod_a and pod_b are required\n")
    r = a.handle("POST", "/api/v1/analyze/pod-communication", b'{"pod_a":"default/x","pod_b":"default/y"}')
    assert r.code == 500 and r.body.startswith(b"Analysis failed: failed to get pod A info")
    assert a.handle("GET", "/api/v1/metrics/nodes/").body == b"Node name is required\n"
    r = a.handle("GET", "/api/v1/metrics/nodes/ghost")
    assert (r.code, r.body) == (404, b"Node not found: metrics not found for node: ghost\n")
    r = a.handle("GET", "/api/v1/metrics/uav/ghost")
    assert (r.code, r.body) == (404, b"UAV not found on node: ghost\n")
    assert a.handle("POST", "/api/v1/uav/report", b"[]").body == b"Invalid JSON body\n"
    assert a.handle("POST", "/api/v1/uav/report", b"{}").body == b"node_name is required\n"
    assert a.handle("GET", "/api/v1//pods").code == 301


def test_success_shapes(mon):
    a = mon.app
    d = J(a.handle("GET", "/api/v1/cluster/status"))
    assert set(d["cluster_info"]) == {"namespaces", "nodes", "pods", "version"} and d["status"] == "success"
    d = J(a.handle("GET", "/api/v1/pods"))
    assert d["count"] == len(d["pods"]) > 5 and set(d["pods"][0]) == {"name", "namespace", "status", "node_name", "ip",
                                                                    "labels", "start_time", "containers"}
    d = J(a.handle("GET", "/api/v1/metrics/nodes"))
    assert set(d) == {"count", "data", "status", "timestamp"} and d["count"] == 3
    node = next(iter(d["data"].values()))
    assert list(node)[:3] == ["node_name", "timestamp", "cpu_capacity"] and "custom_metrics" not in node
    d = J(a.handle("GET", "/api/v1/metrics/snapshot"))
    assert set(d) == {"data", "status"} and set(d["data"]) == {"timestamp", "node_metrics", "pod_metrics",
                                                              "network_metrics", "cluster_metrics"}
    d = J(a.handle("GET", "/api/v1/metrics/pods"))
    assert all("/" in k for k in d["data"])
    d = J(a.handle("GET", "/api/v1/metrics/network"))
    assert d["count"] == 5 and set(d["data"][0]) >= {"source_pod", "target_pod", "connected", "rtt_ms", "test_method"}
    d = J(a.handle("GET", "/api/v1/metrics/uav"))
    e = next(iter(d["data"].values()))
    assert set(e) == {"node_name", "status", "source", "timestamp", "last_heartbeat", "state"} and e["source"] == "pull"
    node = next(iter(d["data"]))
    assert J(a.handle("GET", f"/api/v1/metrics/uav/{node}"))["data"]["node_name"] == node
    d = J(a.handle("POST", "/api/v1/analyze/pod-communication",
                   b'{"pod_a":"default/frontend-5c7d8f9b4-kq2lp","pod_b":"default/nginx-web-6d4cf56db6-8v2mz","explain":false}'))
    assert set(d) == {"analysis", "status", "timestamp"}
    assert list(d["analysis"]) == ["pod_a", "pod_b", "status", "issues", "solutions", "confidence"]


def test_uav_report_to_crd_to_scheduler(mon):
    from k8s_llm_monitor_amd.monitor.cluster.backend import SCHEDULING_REQUESTS
    from k8s_llm_monitor_amd.monitor.scheduler.controller import SchedulerController
    from k8s_llm_monitor_amd.monitor.uav.agent import UAVAgent
    from k8s_llm_monitor_amd.utils import gojson

    a = mon.app
    agent = UAVAgent("edge-1", "10.9.9.9", report_interval_s=10)
    r = a.handle("POST", "/api/v1/uav/report", gojson.dumps(agent.build_report()).encode())
    d = J(r)
    assert d["crd_status"] == "updated" and d["uav_id"] == "UAV-edge-1" and d["heartbeat_interval_seconds"] == 10
    assert J(a.handle("GET", "/api/v1/metrics/uav/edge-1"))["data"]["source"] == "agent"
    crd = J(a.handle("GET", "/api/v1/crd/uav?namespace=all"))
    assert crd["count"] == 1 and crd["data"][0]["spec"]["node_name"] == "edge-1"
    fc = mon.backend
    fc.create(SCHEDULING_REQUESTS, {"metadata": {"name": "job"}, "spec": {"workload": {"name": "w", "namespace": "default"},
                                                                          "minBatteryPercent": 50}}, "default")
    SchedulerController(fc).reconcile()
    st = fc.get(SCHEDULING_REQUESTS, "job", "default")["status"]
    assert st["phase"] == "Assigned" and st["assignedNode"] == "edge-1" and st["assignedUAV"] == "UAV-edge-1"


def test_query_and_analysis_records(mon):
    a = mon.app
    assert a.handle("POST", "/api/v1/query", b"{}").body == b"question is required\n"
    d = J(a.handle("POST", "/api/v1/query", "{\"question\":\"为什么我的pod频繁重启？\"}".encode()))
    assert d["status"] == "success" and d["result"]["question"] == "为什么我的pod频繁重启？" and d["request_id"]
    rec = J(a.handle("GET", f"/api/v1/analysis/{d['request_id']}"))
    assert rec["data"]["request_id"] == d["request_id"]
    d = J(a.handle("POST", "/api/v1/analyze", b'{"type":"anomaly_detection"}'))
    assert d["result"]["type"] == "anomaly_detection"
    assert a.handle("POST", "/api/v1/analyze", b'{"type":"bogus"}').code == 400
    assert J(a.handle("GET", "/api/v1/analysis"))["count"] == 2


def test_real_http_roundtrip(mon):
    srv = make_server(mon.app, "127.0.0.1", 0)
    t = threading.Thread(target=srv.serve_forever, daemon=True)
    t.start()
    try:
        c = http.client.HTTPConnection("127.0.0.1", srv.server_address[1], timeout=10)
        c.request("GET", "/api/v1/metrics/cluster")
        r = c.getresponse()
        body = r.read()
        assert r.status == 200 and r.getheader("Content-Type") == "application/json"
        assert r.getheader("Access-Control-Allow-Origin") == "*" and json.loads(body)["status"] == "success"
        c.request("GET", "/")
        r = c.getresponse()
        assert r.status == 200 and b"K8s LLM Monitor" in r.read()
        c.request("POST", "/api/v1/pods", b"")
        r = c.getresponse()
        assert r.status == 405 and r.read() == b"Method not allowed\n"
        assert r.getheader("X-Content-Type-Options") == "nosniff"
    finally:
        srv.shutdown()


def test_dev_mode_script_without_cluster():
    """scripts/test_with_mock_k8s.sh: the server in development mode (no cluster, no model)."""
    import shutil
    import socket
    import subprocess

    if shutil.which("curl") is None:
        pytest.skip("curl not installed")
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    r = subprocess.run(["bash", "scripts/test_with_mock_k8s.sh", str(port)], capture_output=True, text=True,
                       timeout=120, cwd=os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    assert r.returncode == 0, r.stdout + r.stderr


def test_web_console_pages(mon):
    """W1/W2: both pages are served, every API path they poll answers 200 on a live monitor, and
    the console's status/error bar, manual refresh (with loading state) and UAV/CRD summary card
    are present (reference web/index.html:537-621,796, web/metrics.html:244)."""
    import re

    a = mon.app
    for page in ("/", "/metrics.html"):
        r = a.handle("GET", page)
        assert r.code == 200 and r.ctype.startswith("text/html"), page
    assert a.handle("GET", "/index.html").code == 301  # Go FileServer: /index.html -> ./
    idx = a.handle("GET", "/").body.decode()
    met = a.handle("GET", "/metrics.html").body.decode()
    for needle in ('id="status"', 'id="refresh"', "刷新中…", "活跃 UAV / CRD 记录", 'id="nodeCount"', 'id="podCount"',
                   "errors.push"):
        assert needle in idx, needle
    assert 'id="reload"' in met and 'id="err"' in met and "errs.push" in met
    for path in sorted(set(re.findall(r"'(/api/v1/[a-z/]+)'", idx + met))):
        if path in ("/api/v1/query", "/api/v1/metrics/engine"):  # POST-only / optional (no engine here)
            continue
        assert a.handle("GET", path).code == 200, path


def test_llm_routes_send_analysis_types_to_their_deployment(monkeypatch):
    """``llm.routes`` (models.go:86-90: root_cause on the 70B deployment, anomaly_detection on
    Mixtral): a routed type is generated by the upstream's OpenAI-compatible /v1/chat/completions
    (here a second server of this framework), an unrouted type by the local backend; the prompt is
    built from the local cluster context either way."""
    up_cfg = from_dict({"llm": {"provider": "none"}})
    up = build_monitor(up_cfg, backend=FakeCluster.build(seed=5), start_manager=False, llm=True)
    srv = make_server(up.app, "127.0.0.1", 0)
    t = threading.Thread(target=srv.serve_forever, daemon=True)
    t.start()
    try:
        url = f"http://127.0.0.1:{srv.server_address[1]}/v1"
        monkeypatch.setenv("LLM_ROUTES", f"root_cause={url}")
        cfg = from_dict({"llm": {"provider": "none", "model": "llama-3-70b"}})
        assert cfg.llm.routes == {"root_cause": url}
        m = build_monitor(cfg, backend=FakeCluster.build(seed=2), start_manager=False, llm=True)
        m.manager.collect()
        before = up.app.requests
        d = J(m.app.handle("POST", "/api/v1/analyze", b'{"type":"root_cause"}'))
        assert d["status"] == "success" and d["result"]["type"] == "root_cause"
        assert d["result"]["provider"] == "openai" and d["result"]["model"] == "rule-engine"
        assert up.app.requests == before + 1
        d = J(m.app.handle("POST", "/api/v1/analyze", b'{"type":"anomaly_detection"}'))
        assert d["result"]["provider"] == "rules" and up.app.requests == before + 1
    finally:
        srv.shutdown()


def test_chat_completions_endpoint(mon):
    a = mon.app
    r = a.handle("POST", "/v1/chat/completions", b'{"messages": []}')
    assert r.code == 400
    assert a.handle("GET", "/v1/chat/completions").code == 405
    body = json.dumps({"model": "x", "max_tokens": 16,
                       "messages": [{"role": "user", "content": "节点 n1 状态=NotReady [不健康]"}]}).encode()
    d = J(a.handle("POST", "/v1/chat/completions", body))
    assert d["object"] == "chat.completion" and d["choices"][0]["message"]["role"] == "assistant"
    assert "NotReady" in d["choices"][0]["message"]["content"] and d["usage"]["completion_tokens"] > 0
    # streaming and stop sequences are refused, not silently ignored; top_p passes through
    msgs = [{"role": "user", "content": "hi"}]
    assert a.handle("POST", "/v1/chat/completions", json.dumps({"messages": msgs, "stream": True}).encode()).code == 400
    assert a.handle("POST", "/v1/chat/completions", json.dumps({"messages": msgs, "stop": ["\n"]}).encode()).code == 400
    assert J(a.handle("POST", "/v1/chat/completions", json.dumps({"messages": msgs, "top_p": 0.9}).encode()))["object"]


def test_chat_prompt_fits_the_window():
    """A chat longer than the model window keeps its latest turns (oldest dropped first)."""
    from k8s_llm_monitor_amd.llm.service import AnalysisService

    class Small:
        def max_prompt_tokens(self, max_tokens=None):
            return 300

        def count_tokens(self, text):
            return len(text.encode())

    an = AnalysisService(Small(), max_tokens=16)
    parts = [f"turn {i}: " + "x" * 100 for i in range(10)]
    out = an.fit_chat(parts, 16)
    assert out.endswith(parts[-1]) and "turn 0:" not in out and len(out.encode()) <= 300


def test_context_fits_a_short_model_window():
    """A 1024-token model (GPT-2) with a long cluster context: the service trims the context so the
    prompt leaves room for the requested answer, instead of the engine cutting the prompt's middle
    and leaving room for one token (BASELINE config 1)."""
    from k8s_llm_monitor_amd.engine import EngineConfig, EngineService, LLMEngine
    from k8s_llm_monitor_amd.llm.service import AnalysisService, LocalEngineBackend

    eng = LLMEngine(EngineConfig(model="gpt2-tiny", max_num_seqs=2, max_model_len=512, num_blocks=64, seed=1),
                    device="cpu")
    svc = EngineService(eng)
    try:
        be = LocalEngineBackend(svc, max_tokens=32, temperature=0.0, timeout_s=60.0)
        assert be.max_len == 512
        an = AnalysisService(be, max_tokens=32)
        ctx = "\n".join(f"- node-{i:03d} CPU={i % 97}% MEM={i % 89}% pods={i % 31}" for i in range(400))
        assert be.count_tokens(ctx) > 512
        r = an.query("哪个节点最忙?", max_tokens=32, ignore_eos=True, context_text=ctx)
        assert r.status == "success", r.error
        assert r.result["completion_tokens"] == 32 and r.result["finish_reason"] == "length"
        assert r.result["prompt_tokens"] + 32 <= 512
    finally:
        svc.close()


def test_record_store_keeps_answers_and_reads_back_plain(tmp_path):
    """RecordStore keeps a finished AnalysisResponse as is (no Go-JSON round trip on the answer's
    path) and converts on read: get / list return the same plain dicts the round trip produced, and
    the file store writes one Go-JSON line per record."""
    from k8s_llm_monitor_amd.llm.service import RecordStore
    from k8s_llm_monitor_amd.monitor.types import AnalysisResponse
    from k8s_llm_monitor_amd.utils import gojson
    from k8s_llm_monitor_amd.utils.gojson import utcnow

    for kind in ("memory", "file"):
        st = RecordStore(kind, path=str(tmp_path / kind), capacity=2)
        rs = [AnalysisResponse(request_id=f"r{i}", status="success",
                               result={"type": "query", "answer": f"a<{i}>", "latency_ms": 12.5 + i},
                               timestamp=utcnow()) for i in range(3)]
        for r in rs:
            st.put(r)
        assert st.get("r0") is None  # capacity 2: the oldest was evicted
        assert st.get("r2") == gojson.to_plain(rs[2])
        assert st.list(10) == [gojson.to_plain(rs[1]), gojson.to_plain(rs[2])]
        if kind == "file":
            lines = (tmp_path / kind / "analysis_records.jsonl").read_text().splitlines()
            assert [json.loads(x)["request_id"] for x in lines] == ["r0", "r1", "r2"]


def test_gojson_float_fast_path_matches_decimal_form():
    """format_float's fixed-point fast path (repr already in Go's digits) equals the Decimal form
    it replaced, over random values across the fixed-point range and integral floats."""
    import random
    from decimal import Decimal

    from k8s_llm_monitor_amd.utils.gojson import format_float

    def slow(f):
        s = format(Decimal(repr(f)), "f")
        return s.rstrip("0").rstrip(".") if "." in s else s

    r = random.Random(0)
    for _ in range(20000):
        f = r.choice([r.uniform(-1e3, 1e3), 10 ** r.uniform(-6, 20.9) * r.choice([1, -1]),
                      float(r.randint(-10 ** 6, 10 ** 6)), round(r.uniform(0, 100), 2)])
        if f != 0:
            assert format_float(f) == slow(f), f


@pytest.mark.parametrize("inline", [True, False])
def test_query_answer_budget_timeout_is_504(mon, inline):
    """A backend whose answer budget runs out answers /api/v1/query with 504, both when the query
    runs in the handler thread (the backend bounds its own wait: ``enforces_deadline``) and on the
    bounded pool."""
    from concurrent.futures import TimeoutError as FutTimeout

    class SlowBackend:
        provider, model = "stub", "stub"
        enforces_deadline = inline

        def count_tokens(self, text):
            return len(text) // 4

        def generate(self, prompt, **kw):
            if inline:  # the engine backend's own budget (LocalEngineBackend.generate)
                raise AnswerBudgetExceeded("answer not ready within the answer budget")
            time.sleep(3)  # the pool's write-timeout backstop (1 s here) fires first

    from k8s_llm_monitor_amd.llm.service import AnswerBudgetExceeded

    a = mon.app
    a.write_timeout_s = a.llm_timeout_s = 1.5
    a.analysis.backend = SlowBackend()
    r = a.handle("POST", "/api/v1/query", json.dumps({"question": "why is node-1 NotReady?"}).encode())
    assert r.code == 504, (r.code, r.body[:200])
    assert FutTimeout is not None


def test_routed_socket_timeout_is_an_error_record_not_504(mon):
    """only the engine's own answer budget (AnswerBudgetExceeded) means 504.  A routed
    backend's socket timeout - a builtin TimeoutError, the same class as the futures one on
    Python >= 3.11 - becomes an error record (500 with the record), on every interpreter."""
    class Upstream:
        provider, model = "openai", "upstream"

        def generate(self, prompt, **kw):
            raise TimeoutError("timed out")

    a = mon.app
    a.analysis.routes["query"] = Upstream()
    r = a.handle("POST", "/api/v1/query", json.dumps({"question": "why?", "context": {"cluster_state": "x"}}).encode())
    assert r.code == 500, (r.code, r.body[:200])
    d = J(r)
    assert d["status"] == "error" and "TimeoutError" in d["error"]


def test_fit_uses_the_routed_backends_window(mon):
    """a routed analysis type is trimmed to ITS backend's window with ITS tokenizer; a
    backend that publishes no window gets the context untrimmed."""
    class Small:
        provider, model = "stub", "small"
        seen = []

        def max_prompt_tokens(self, max_tokens=None):
            return 200

        def count_tokens(self, text):
            return len(text.encode())

        def generate(self, prompt, **kw):
            self.seen.append(prompt)
            return {"text": "ok", "model": self.model, "provider": self.provider}

    class NoWindow(Small):
        max_prompt_tokens = None

    ctx = "\n".join(f"- node-{i:03d} CPU={i % 97}%" for i in range(400))
    a = mon.app
    small, big = Small(), NoWindow()
    small.seen, big.seen = [], []
    a.analysis.routes["query"] = small
    J(a.handle("POST", "/api/v1/query", json.dumps({"question": "q", "context": {"cluster_state": ctx}}).encode()))
    assert len(small.seen[-1].encode()) < 400
    a.analysis.routes["query"] = big
    J(a.handle("POST", "/api/v1/query", json.dumps({"question": "q", "context": {"cluster_state": ctx}}).encode()))
    assert ctx in big.seen[-1]


def test_query_runs_inline_only_with_a_ready_context(mon, monkeypatch):
    """the handler-thread (inline) path skips the write-timeout backstop, so it is taken
    only when building the prompt cannot block on the K8s API: a supplied context or a context
    already built for the current snapshot; otherwise the bounded pool runs the query."""
    from k8s_llm_monitor_amd.monitor import server as S

    class Eng:
        provider, model = "stub", "stub"
        enforces_deadline = True

        def count_tokens(self, text):
            return 1

        def generate(self, prompt, **kw):
            return {"text": "ok", "model": self.model, "provider": self.provider}

    used = []
    real = S._bounded_pool

    def spy():
        used.append(1)
        return real()

    monkeypatch.setattr(S, "_bounded_pool", spy)
    a = mon.app
    a.analysis.backend = Eng()
    a.analysis._ctx_cache = (None, "")  # a new snapshot: its context is not built yet
    assert not a.analysis.context_ready()
    assert J(a.handle("POST", "/api/v1/query", b'{"question":"q"}'))["status"] == "success"
    assert used == [1]  # pool path
    assert a.analysis.context_ready()  # built by that query
    J(a.handle("POST", "/api/v1/query", b'{"question":"q"}'))
    J(a.handle("POST", "/api/v1/query", b'{"question":"q","context":{"cluster_state":"c"}}'))
    assert used == [1]  # both inline
