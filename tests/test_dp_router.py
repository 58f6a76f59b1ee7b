"""Data-parallel serving: the least-loaded router over engine replica processes (engine/dp.py)."""
import concurrent.futures as cf

import pytest

from k8s_llm_monitor_amd.engine import EngineConfig, LLMEngine, SamplingParams
from k8s_llm_monitor_amd.engine.dp import ReplicaRouter

CFG = dict(model="llama-tiny", max_num_seqs=4, max_model_len=256, num_blocks=64, use_graphs=False, seed=7,
           dtype="float32")


def test_router_spreads_requests_and_matches_single_engine():
    prompts = [f"pod-{i} CrashLoopBackOff in namespace default, 为什么?" for i in range(6)]
    sp = SamplingParams(max_tokens=4, temperature=0.0, ignore_eos=True)
    ref = [s.output_ids for s in LLMEngine(EngineConfig(**CFG), device="cpu").generate(prompts, sp)]
    router = ReplicaRouter(EngineConfig(**CFG), ["cpu", "cpu"])
    try:
        futs = [router.submit(p, sp, request_id=f"r{i}") for i, p in enumerate(prompts)]
        outs = [f.result(timeout=120) for f in futs]
        assert [seq.output_ids for _, seq in outs] == ref  # same model in every replica
        assert {seq.replica for _, seq in outs} == {0, 1}  # both replicas served
        assert all(seq.timings()["completion_tokens"] == 4 for _, seq in outs)
        st = router.stats()
        assert st["dp_replicas"] == 2 and st["healthy"] and st["finished"] == 6
        assert [r["outstanding"] for r in st["replicas"]] == [0, 0]
        assert router.engine.model_cfg.name == "llama-tiny"
    finally:
        router.close()
    assert all(not r.proc.is_alive() for r in router.replicas)


def test_router_backs_local_engine_backend_concurrently():
    from k8s_llm_monitor_amd.llm.service import LocalEngineBackend

    router = ReplicaRouter(EngineConfig(**CFG), ["cpu", "cpu"])
    try:
        be = LocalEngineBackend(router, max_tokens=3, temperature=0.0, timeout_s=120)
        with cf.ThreadPoolExecutor(8) as ex:
            res = list(ex.map(lambda i: be.generate(f"node-{i} NotReady", ignore_eos=True), range(8)))
        assert all(r["completion_tokens"] == 3 and r["provider"] == "local-rocm" for r in res)
        # streaming through the router: the replica forwards token batches over its pipe
        items = list(be.stream("node-9 NotReady", max_tokens=5, ignore_eos=True))
        final = items[-1]
        assert final["completion_tokens"] == 5
        assert "".join(x for x in items[:-1] if isinstance(x, str)) == final["text"]
        # a streaming consumer that goes away cancels the request in its replica
        be_long = LocalEngineBackend(router, max_tokens=200, temperature=0.0, timeout_s=120)
        g = be_long.stream("node-10 NotReady " * 8, ignore_eos=True)
        assert next(x for x in g if isinstance(x, str))
        g.close()
        import time

        t0 = time.time()
        while sum(r.get("cancelled", 0) for r in router.stats()["replicas"]) < 1 and time.time() - t0 < 30:
            time.sleep(0.05)
        assert sum(r.get("cancelled", 0) for r in router.stats()["replicas"]) == 1
    finally:
        router.close()


def test_server_assembly_with_dp_replicas(tmp_path):
    from k8s_llm_monitor_amd.monitor.app import make_llm_backend
    from k8s_llm_monitor_amd.monitor.config import load

    p = tmp_path / "config.yaml"
    p.write_text("llm:\n  provider: local-rocm\n  model: llama-tiny\n  dp_replicas: 2\n  max_batch: 4\n"
                 "  max_model_len: 256\n  kv_cache_gb: 0.01\n  use_graphs: false\n  max_tokens: 3\n")
    cfg = load(str(p))
    backend, eng, svc = make_llm_backend(cfg)
    try:
        assert eng is None and len(svc.replicas) == 2
        r = backend.generate("kube-system coredns CrashLoopBackOff", ignore_eos=True)
        assert r["completion_tokens"] == 3
    finally:
        svc.close()


@pytest.mark.gpu
def test_gpu_router_two_replicas_share_one_gpu():
    """Two replica processes on cuda:0 (the box has one GPU): HIP kernels + hipGraph decode in
    each child, answers equal a single in-process engine's."""
    cfg = dict(model="llama-tiny-d128", max_num_seqs=8, max_model_len=1024, num_blocks=256, seed=3)
    prompts = ["why is pod default/api not ready?", "node-003 NotReady 为什么", "coredns CrashLoopBackOff"] * 2
    sp = SamplingParams(max_tokens=6, temperature=0.0, ignore_eos=True)
    eng = LLMEngine(EngineConfig(**cfg), device="cuda:0")
    eng.warmup()
    ref = [s.output_ids for s in eng.generate(prompts, sp)]
    router = ReplicaRouter(EngineConfig(**cfg), ["cuda:0", "cuda:0"], start_timeout_s=300)
    try:
        outs = [f.result(timeout=120) for f in [router.submit(p, sp) for p in prompts]]
        assert [seq.output_ids for _, seq in outs] == ref
        assert {seq.replica for _, seq in outs} == {0, 1}
    finally:
        router.close()
