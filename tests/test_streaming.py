"""Token streaming: engine per-request token callbacks, the incremental detokenizer, and
``POST /api/v1/query {"stream": true}`` as Server-Sent Events over chunked HTTP/1.1."""
import http.client
import json

import pytest

from k8s_llm_monitor_amd.engine import EngineConfig, EngineService, LLMEngine, SamplingParams
from k8s_llm_monitor_amd.engine.tokenizer import tokenizer_for
from k8s_llm_monitor_amd.llm.service import IncrementalDetokenizer
from k8s_llm_monitor_amd.models.config import get_config


def test_incremental_detokenizer_multibyte():
    tok = tokenizer_for(get_config("llama-3-8b"))
    text = "集群状态概览: node-001 CPU=93.1% [资源压力] 为什么我的pod频繁重启？ 🚀 done"
    ids = tok.encode(text, bos=False)
    det = IncrementalDetokenizer(tok)
    out = []
    for t in ids:  # one token at a time, as a decode step delivers them
        d = det.add([t])
        assert "�" not in d
        out.append(d)
    out.append(det.flush())
    assert "".join(out) == tok.decode(ids) == text


@pytest.fixture(scope="module")
def engine_service():
    eng = LLMEngine(EngineConfig(model="llama-tiny", max_num_seqs=4, max_model_len=1024, num_blocks=256,
                                 use_graphs=False, seed=3), device="cpu")
    svc = EngineService(eng)
    yield svc
    svc.close()


def test_engine_service_streams_every_token_in_order(engine_service):
    got = []
    fut = engine_service.submit("pod default/api CrashLoopBackOff", SamplingParams(max_tokens=9, temperature=0.0,
                                                                                    ignore_eos=True),
                                on_tokens=got.append)
    text, seq = fut.result(timeout=120)
    flat = [t for chunk in got for t in chunk]
    assert flat == seq.output_ids and len(flat) == 9
    plain, seq2 = engine_service.submit("pod default/api CrashLoopBackOff",
                                        SamplingParams(max_tokens=9, temperature=0.0, ignore_eos=True)).result(120)
    assert seq2.output_ids == seq.output_ids  # streaming does not change the answer


def test_query_stream_over_http():
    from k8s_llm_monitor_amd.monitor.app import build_app_for_bench

    eng = LLMEngine(EngineConfig(model="llama-tiny", max_num_seqs=4, max_model_len=8192, num_blocks=2048,
                                 use_graphs=False, seed=1), device="cpu")
    svc = EngineService(eng)
    srv, port = build_app_for_bench(svc)
    try:
        body = json.dumps({"question": "为什么我的pod频繁重启？", "max_tokens": 7, "ignore_eos": True, "stream": True,
                           "context": {"cluster_state": "node-001 CPU=93.1% [资源压力]"}})
        conn = http.client.HTTPConnection("127.0.0.1", port, timeout=300)
        conn.request("POST", "/api/v1/query", body, {"Content-Type": "application/json"})
        r = conn.getresponse()
        assert r.status == 200
        assert r.getheader("Content-Type") == "text/event-stream"
        assert r.getheader("Transfer-Encoding") == "chunked"
        raw = r.read().decode()  # http.client de-chunks
        conn.close()
        events = [e for e in raw.split("\n\n") if e.strip()]
        deltas, done = [], None
        for e in events:
            lines = e.split("\n")
            if lines[0] == "event: done":
                done = json.loads(lines[1][len("data: "):])
            else:
                deltas.append(json.loads(lines[0][len("data: "):])["delta"])
        assert done is not None and done["status"] == "success"
        assert done["result"]["completion_tokens"] == 7
        assert "".join(deltas) == done["result"]["answer"]
        # the streamed record is stored like a synchronous one
        conn = http.client.HTTPConnection("127.0.0.1", port, timeout=60)
        conn.request("GET", f"/api/v1/analysis/{done['request_id']}")
        rec = json.loads(conn.getresponse().read())
        conn.close()
        assert rec["status"] == "success" and rec["data"]["request_id"] == done["request_id"]
    finally:
        svc.close()
        srv.shutdown()


def test_cancel_frees_the_sequence(engine_service):
    eng = engine_service.engine
    free0 = eng.sched.blocks.num_free
    got = []
    fut = engine_service.submit("node-003 NotReady " * 20, SamplingParams(max_tokens=400, temperature=0.0,
                                                                          ignore_eos=True), on_tokens=got.append)
    import time

    t0 = time.time()
    while not got and time.time() - t0 < 60:  # wait until it is decoding
        time.sleep(0.01)
    assert got
    assert engine_service.cancel(fut) and fut.cancelled()
    t0 = time.time()
    while (eng.sched.running or eng.sched.waiting) and time.time() - t0 < 30:
        time.sleep(0.01)
    assert not eng.sched.running and not eng.sched.waiting
    assert eng.sched.blocks.num_free == free0  # its KV blocks went back to the pool
    assert engine_service.stats()["cancelled"] >= 1
    # the engine keeps serving
    text, seq = engine_service.submit("ok?", SamplingParams(max_tokens=3, temperature=0.0,
                                                            ignore_eos=True)).result(60)
    assert len(seq.output_ids) == 3


def test_stream_consumer_going_away_cancels(engine_service):
    from k8s_llm_monitor_amd.llm.service import LocalEngineBackend

    be = LocalEngineBackend(engine_service, max_tokens=500, temperature=0.0, timeout_s=60)
    before = engine_service.stats()["cancelled"]
    g = be.stream("pod default/db OOMKilled " * 10, ignore_eos=True)
    first = next(x for x in g if isinstance(x, str))
    assert first
    g.close()  # what the HTTP handler does when the client disconnects
    import time

    t0 = time.time()
    while engine_service.stats()["cancelled"] == before and time.time() - t0 < 30:
        time.sleep(0.01)
    assert engine_service.stats()["cancelled"] == before + 1


def test_prometheus_metrics_endpoint(engine_service):
    from k8s_llm_monitor_amd.monitor.cluster.client import K8sClient
    from k8s_llm_monitor_amd.monitor.cluster.fake import FakeCluster
    from k8s_llm_monitor_amd.monitor.config import from_dict
    from k8s_llm_monitor_amd.monitor.metrics.manager import ManagerConfig, MetricsManager
    from k8s_llm_monitor_amd.monitor.server import MonitorApp

    fake = FakeCluster.build(seed=0)
    cfg = from_dict({})
    mgr = MetricsManager(fake, ManagerConfig(namespaces=["default"]))
    mgr.collect()
    app = MonitorApp(K8sClient(fake, cfg.k8s), mgr, None, engine_service)
    r = app.handle("GET", "/metrics")
    assert r.code == 200 and r.ctype.startswith("text/plain; version=0.0.4")
    text = r.body.decode()
    assert "# TYPE k8sllm_engine_generated_tokens_total counter" in text
    assert 'k8sllm_engine_healthy{model="llama-tiny"} 1' in text
    assert "k8sllm_cluster_total_nodes " in text and "k8sllm_http_requests_total 1" in text
    for line in text.splitlines():  # every sample line is `name[{labels}] number`
        if not line.startswith("#"):
            float(line.rsplit(" ", 1)[1])
    assert app.handle("POST", "/metrics").code == 405


@pytest.mark.gpu
def test_gpu_streaming_and_cancel_with_graphs():
    """Token streaming and cancellation on the GPU engine (hipGraph decode, pipelined readback)."""
    import time

    import torch

    from k8s_llm_monitor_amd import ops

    ops.native()
    eng = LLMEngine(EngineConfig(model="llama-tiny-d128", max_num_seqs=8, max_model_len=1024, num_blocks=256,
                                 seed=0), device="cuda:0")
    eng.warmup()
    svc = EngineService(eng)
    try:
        sp = SamplingParams(max_tokens=24, temperature=0.0, ignore_eos=True)
        got = []
        text, seq = svc.submit("pod default/api CrashLoopBackOff", sp, on_tokens=got.append).result(120)
        assert [t for c in got for t in c] == seq.output_ids and len(seq.output_ids) == 24
        _, seq2 = svc.submit("pod default/api CrashLoopBackOff", sp).result(120)
        assert seq2.output_ids == seq.output_ids
        free0 = eng.sched.blocks.num_free
        got = []
        fut = svc.submit("node-003 NotReady " * 10, SamplingParams(max_tokens=900, temperature=0.0, ignore_eos=True),
                         on_tokens=got.append)
        t0 = time.time()
        while not got and time.time() - t0 < 60:
            time.sleep(0.005)
        assert svc.cancel(fut)
        t0 = time.time()
        while (eng.sched.running or eng.sched.waiting) and time.time() - t0 < 30:
            time.sleep(0.005)
        assert eng.sched.blocks.num_free == free0
        _, seq3 = svc.submit("pod default/api CrashLoopBackOff", sp).result(120)
        assert seq3.output_ids == seq.output_ids  # no state leaked from the cancelled request
        torch.cuda.synchronize()
    finally:
        svc.close()
