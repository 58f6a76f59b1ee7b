"""The HTTP paths bench.py drives, end to end on the CPU with a tiny model: POST /api/v1/query
and POST /api/v1/analyze/pod-communication (LLM explanation) through the in-process server, the
engine thread and continuous batching."""
import os
import threading

import pytest

from k8s_llm_monitor_amd.engine import EngineConfig, EngineService, LLMEngine
from k8s_llm_monitor_amd.llm.synthetic import synthetic_context
from k8s_llm_monitor_amd.monitor.app import (bench_pod_pairs, build_app_for_bench, post_pod_communication,
                                             post_queries)


@pytest.fixture(scope="module")
def served():
    eng = LLMEngine(EngineConfig(model="llama-tiny", max_num_seqs=8, max_model_len=8192, num_blocks=2048,
                                 use_graphs=False, seed=1), device="cpu")
    svc = EngineService(eng)
    srv, port = build_app_for_bench(svc)
    yield svc, port
    svc.close()
    srv.shutdown()


def test_query_path(served):
    svc, port = served
    # llama-tiny's 1024-position window: keep the synthetic cluster context short
    items = [(q, ctx[:500]) for ctx, q in (synthetic_context(s) for s in range(3))]
    res = post_queries(port, items, 6)
    assert len(res) == 3
    assert all(r["completion_tokens"] == 6 and r["prompt_tokens"] > 100 for r in res)


def test_query_path_from_loadgen_process(served):
    """The bench's default client: a child load-generator process posting the wave."""
    from k8s_llm_monitor_amd.monitor.loadgen import LoadGen

    svc, port = served
    lg = LoadGen(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    try:
        items = [(q, ctx[:400]) for ctx, q in (synthetic_context(s) for s in range(10, 13))]
        res = lg.post_queries(port, items, 4)
        assert len(res) == 3 and all(r["completion_tokens"] == 4 and r["http_latency_ms"] > 0 for r in res)
        res = lg.post_pod_communication(port, bench_pod_pairs(2), 3)
        assert len(res) == 2 and all(r["completion_tokens"] == 3 for r in res)
        with pytest.raises(RuntimeError, match="unknown op"):
            lg._call({"op": "bogus"})  # errors come back to the parent; the child keeps serving
        assert len(lg.post_queries(port, items[:1], 2)) == 1
        # staged payloads: only the key crosses the pipe; the same keep-alive client serves twice
        lg.stage("w0", items)
        for _ in range(2):
            res = lg.post_queries(port, None, 3, staged="w0", slim=True)
            assert [r["completion_tokens"] for r in res] == [3, 3, 3]
            assert set(res[0]) <= {"http_status", "http_latency_ms", "t_send_s", "error", "prompt_tokens",
                                   "completion_tokens", "ttft_ms", "latency_ms", "finish_reason", "type"}
    finally:
        lg.close()
    assert lg.proc.returncode == 0


def test_query_client_keeps_connections(served):
    """Consecutive waves reuse each worker's HTTP/1.1 connection (no reconnect per request)."""
    from k8s_llm_monitor_amd.monitor.app import QueryClient

    svc, port = served
    cl = QueryClient(workers=2)
    try:
        items = [(q, ctx[:300]) for ctx, q in (synthetic_context(s) for s in range(20, 22))]

        def conns() -> set:
            # one probe per worker thread (a barrier holds each worker until both have one), so
            # every worker's connection is seen, whichever worker served the wave's requests
            bar = threading.Barrier(2)

            def probe():
                bar.wait(timeout=10)
                return getattr(cl._tls, "conn", None)

            fs = [cl.ex.submit(probe) for _ in range(2)]
            return {id(c) for c in (f.result() for f in fs) if c is not None}

        cl.post_queries(port, items, 2)
        before = conns()
        cl.post_queries(port, items, 2)
        after = conns()
        assert before and before & after
    finally:
        cl.close()


def test_pod_communication_path(served):
    svc, port = served
    pairs = bench_pod_pairs(3)
    assert all("/" in a and "/" in b for a, b in pairs)
    res = post_pod_communication(port, pairs, 5)
    assert len(res) == 3
    assert all(r["completion_tokens"] == 5 and r["type"] == "pod_communication" for r in res)


@pytest.mark.parametrize("n", [2, 8])
def test_bench_ranks_under_torchrun_cpu(n):
    """The driver's multi-GPU contract rehearsed on CPU: torchrun, n ranks (gloo; 8 = the scaling
    run's largest point), one JSON line from rank 0 with the whole-job value, n_gpus n and dp<n>
    parallelism."""
    import json
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    batch = 4 if n == 2 else 2

    # --standalone: torchrun binds its own rendezvous store on a port the OS picks (no probed port
    # that another process can take before the launch); 127.0.0.1 as the task's rendezvous rule asks
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--standalone", "--local-addr", "127.0.0.1",
                        "--nnodes=1", "--nproc-per-node", str(n), "bench.py", "--gpus", str(n), "--steps", "1",
                        "--warmup", "1", "--model", "llama-tiny", "--batch", str(batch), "--max-new-tokens", "4"],
                       capture_output=True, text=True, timeout=600, cwd=root, env={**os.environ, "OMP_NUM_THREADS": "1"})
    if r.returncode != 0:  # keep the failing ranks' stderr for the record (no relaunch)
        os.makedirs(os.path.join(root, "gpurun_out"), exist_ok=True)
        with open(os.path.join(root, "gpurun_out", f"torchrun_{n}_ranks_failure.err"), "w") as f:
            f.write(r.stderr)
    assert r.returncode == 0, r.stderr[-4000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    d = json.loads(lines[0])
    assert d["n_gpus"] == n and d["config"]["parallelism"] == f"dp{n}" and d["config"]["global_batch"] == n * batch
    assert d["steps"] == 1 and d["warmup"] == 1 and d["value"] > 0 and d["scaling"] == "weak"
    assert d["config"]["path"] == "http" and d["config"]["client"] == "process"


def _bench(args):
    import json
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, "bench.py", *args], capture_output=True, text=True, timeout=400, cwd=root,
                       env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    return json.loads(lines[0])


@pytest.mark.parametrize("tp", [1, 2])
def test_bench_self_launches_ranks_cpu(tp):
    """``python bench.py --gpus 2`` with no torchrun: the parent spawns the 2 ranks itself (DP
    replicas, or one TP=2 replica whose worker mirrors the leader over the shared-memory step bus)."""
    d = _bench(["--gpus", "2", "--tp", str(tp), "--steps", "1", "--warmup", "1", "--model", "llama-tiny",
                "--batch", "3", "--max-new-tokens", "3"])
    assert d["n_gpus"] == 2 and d["dist"]["world_size"] == 2 and d["dist"]["tp"] == tp
    assert d["config"]["parallelism"] == ("dp2" if tp == 1 else "tp2")
    assert d["config"]["global_batch"] == (6 if tp == 1 else 3)
    assert d["value"] > 0 and "TP=%d" % tp in d["metric"]
    if tp == 2:
        assert d["dist"]["step_bus"] == "ShmStepBus"


def test_bench_open_loop_and_latency_modes_cpu():
    d = _bench(["--steps", "1", "--warmup", "0", "--model", "llama-tiny", "--mode", "poisson", "--rate", "50",
                "--batch", "4", "--max-new-tokens", "4", "--production"])
    assert d["config"]["mode"] == "poisson" and d["requests"]["ok_rank0"] == 4
    assert d["ttft_ms"]["p50"] is not None and d["config"]["server_timeouts"].startswith("production")
    d = _bench(["--steps", "2", "--warmup", "0", "--model", "llama-tiny", "--mode", "latency",
                "--max-new-tokens", "3"])
    assert d["config"]["global_batch"] == 1 and d["steps"] == 2 and d["p50_latency_ms"] > 0
