"""Data-parallel serving: one engine replica process per GPU behind a least-loaded request router
(SURVEY.md §2.10 "DP: one independent TP=1 engine per GPU; the request router in the control
plane load-balances"; ``llm.dp_replicas``).

The server process owns the HTTP front end and the router and never touches a GPU; replica ``i``
is a spawned child process that builds its own ``LLMEngine`` on ``devices[i]`` (the same model -
same config and seed - with its own KV cache, hipGraphs and continuous-batching queue) and serves
requests over a pipe.  Requests and answers are small (prompt text in, generated text + timings
out), so the router adds ~0.1 ms per request and nothing to the GPU path; each replica batches
whatever it is given, and the router keeps the per-replica outstanding counts level so the
replicas' batches stay equally full.

``ReplicaRouter`` is a drop-in for ``EngineService`` (``submit`` -> Future of ``(text, seq)``,
``stats``, ``close``, ``engine.model_cfg`` / ``engine.tokenizer``), so ``LocalEngineBackend`` and
the REST handlers work unchanged.  Children are started with the ``spawn`` method before anything
in this process initialises a GPU, and every replica is joined on ``close``.
"""
from __future__ import annotations

import itertools
import multiprocessing as mp
import threading
import time
from collections import deque
from concurrent.futures import Future
from dataclasses import asdict
from typing import Optional, Sequence as Seq, Union

from .sequence import SamplingParams


class RemoteSeq:
    """What callers read of a finished sequence, rebuilt from a replica's answer."""

    def __init__(self, d: dict):
        self._timings = d["timings"]
        self.finish_reason = d.get("finish_reason")
        self.output_ids = d.get("output_ids", [])
        self.prompt_ids = d.get("prompt_ids", [])
        self.replica = d.get("replica")

    def timings(self) -> dict:
        return dict(self._timings)


class _EngineInfo:
    """``router.engine``: the model config and tokenizer (built locally, CPU only) - resolved
    exactly as each replica's LLMEngine resolves them (engine.py), so token counts and streamed
    detokenization use the replicas' vocabulary: a Hugging Face ``weights`` directory wins over
    the built-in model name."""

    def __init__(self, model: str, overrides: dict, weights: Optional[str] = None, cfg=None):
        from ..models.checkpoint import config_from_hf
        from ..models.config import get_config
        from .tokenizer import tokenizer_for, tokenizer_from_dir

        mc = config_from_hf(weights) if weights else get_config(model)
        if overrides:
            mc = mc.replace(**overrides)
        self.model_cfg = mc
        self.cfg = cfg
        self.tokenizer = tokenizer_from_dir(weights, mc) if weights else tokenizer_for(mc)


def _replica_main(conn, idx: int, cfg: dict, device: str) -> None:
    """Child process: one engine replica serving the router's pipe until ``close``."""
    import torch

    from .engine import EngineConfig, EngineOverloaded, EngineService, EngineUnavailable, LLMEngine

    try:
        if device.startswith("cuda"):
            torch.cuda.set_device(torch.device(device))
        eng = LLMEngine(EngineConfig(**cfg), device=device)
        eng.warmup()
        svc = EngineService(eng)
    except BaseException as e:  # noqa: BLE001 - report and exit
        conn.send(("error", -1, repr(e)))
        return
    conn.send(("ready", -1, {"device": device, "init_s": round(eng.init_s, 2)}))
    send_lock = threading.Lock()

    def send(msg) -> None:
        with send_lock:
            conn.send(msg)

    live: dict = {}  # key -> local future of requests still running

    def on_done(key: int, fut: Future) -> None:
        if fut.cancelled():
            send(("fail", key, "cancelled"))
            return
        try:
            text, seq = fut.result()
            send(("done", key, {"text": text, "timings": seq.timings(), "finish_reason": seq.finish_reason,
                                "output_ids": list(seq.output_ids), "prompt_ids": list(seq.prompt_ids),
                                "replica": idx}))
        except (EngineOverloaded, EngineUnavailable) as e:
            send(("busy", key, str(e)))
        except BaseException as e:  # noqa: BLE001
            send(("fail", key, repr(e)))

    while True:
        try:
            kind, key, body = conn.recv()
        except EOFError:
            break
        if kind == "req":
            prompt, params, rid, stream, budget = (tuple(body) + (False, None))[:5]
            cb = (lambda ids, k=key: send(("tok", k, ids))) if stream else None
            deadline = time.perf_counter() + budget if budget is not None else None
            fut = svc.submit(prompt, SamplingParams(**params), rid, on_tokens=cb, deadline=deadline)
            live[key] = fut
            fut.add_done_callback(lambda f, k=key: (live.pop(k, None), on_done(k, f)))
        elif kind == "cancel":
            f = live.get(key)
            if f is not None:
                svc.cancel(f)
        elif kind == "stats":
            send(("stats", key, svc.stats()))
        elif kind == "close":
            break
    svc.close()
    send(("closed", -1, None))


class _Replica:
    def __init__(self, idx: int, proc, conn, device: str):
        self.idx, self.proc, self.conn, self.device = idx, proc, conn, device
        self.outstanding = 0
        self.submitted = 0
        self.info: dict = {}
        self.reader: Optional[threading.Thread] = None
        self.send_lock = threading.Lock()

    def send(self, msg) -> None:
        with self.send_lock:
            self.conn.send(msg)


class ReplicaRouter:
    """Least-outstanding-requests router over ``n`` engine replica processes."""

    def __init__(self, engine_cfg, devices: Seq[str], start_timeout_s: float = 900.0):
        from .engine import EngineConfig

        assert isinstance(engine_cfg, EngineConfig)
        if not devices:
            raise ValueError("ReplicaRouter needs at least one device")
        self.engine = _EngineInfo(engine_cfg.model, engine_cfg.model_overrides, engine_cfg.weights, engine_cfg)
        self._keys = itertools.count()
        self._pending: dict = {}
        self._streams: dict = {}  # key -> on_tokens of streaming requests
        self._lock = threading.Lock()
        self._error: Optional[str] = None
        self.latencies_ms: deque = deque(maxlen=4096)
        ctx = mp.get_context("spawn")
        cfg = asdict(engine_cfg)
        self.replicas: list[_Replica] = []
        for i, dev in enumerate(devices):
            parent, child = ctx.Pipe()
            p = ctx.Process(target=_replica_main, args=(child, i, cfg, dev),
                            name=f"llm-replica-{i}", daemon=True)
            p.start()
            child.close()
            self.replicas.append(_Replica(i, p, parent, dev))
        deadline = time.time() + start_timeout_s
        for r in self.replicas:  # wait for every replica to build its engine and capture its graphs
            if not r.conn.poll(max(0.0, deadline - time.time())):
                self.close()
                raise RuntimeError(f"replica {r.idx} ({r.device}) did not start in {start_timeout_s:.0f} s")
            kind, _, body = r.conn.recv()
            if kind != "ready":
                self.close()
                raise RuntimeError(f"replica {r.idx} ({r.device}) failed: {body}")
            r.info = body
        for r in self.replicas:
            r.reader = threading.Thread(target=self._read, args=(r,), name=f"replica-reader-{r.idx}", daemon=True)
            r.reader.start()

    # ------------------------------------------------------------------ EngineService API
    @property
    def healthy(self) -> bool:
        return self._error is None and all(r.proc.is_alive() for r in self.replicas)

    def submit(self, prompt: Union[str, list], params: Optional[SamplingParams] = None,
               request_id: Optional[str] = None, on_tokens=None, deadline: Optional[float] = None) -> Future:
        """As EngineService.submit; ``on_tokens`` is called on the router's reader thread with the
        token ids the replica streams back (``tok`` messages) before the answer arrives."""
        fut: Future = Future()
        if self._error is not None:
            fut.set_exception(RuntimeError(f"replica failed: {self._error}"))
            return fut
        p = asdict(params or SamplingParams())
        p["stop_token_ids"] = tuple(p["stop_token_ids"])
        key = next(self._keys)
        with self._lock:
            r = min(self.replicas, key=lambda x: (x.outstanding, x.submitted))
            r.outstanding += 1
            r.submitted += 1
            self._pending[key] = (fut, r)
            if on_tokens is not None:
                self._streams[key] = on_tokens
        budget = deadline - time.perf_counter() if deadline is not None else None  # replica clocks differ
        r.send(("req", key, (prompt, p, request_id, on_tokens is not None, budget)))
        return fut

    def cancel(self, fut: Future) -> bool:
        """Abort a submitted request (its replica drops the sequence and frees its KV)."""
        with self._lock:
            key = next((k for k, (f, _) in self._pending.items() if f is fut), None)
            rep = self._pending[key][1] if key is not None else None
        if key is None or not fut.cancel():
            return False
        rep.send(("cancel", key, None))
        return True

    def _read(self, r: _Replica) -> None:
        while True:
            try:
                kind, key, body = r.conn.recv()
            except (EOFError, OSError):
                break
            if kind == "tok":
                cb = self._streams.get(key)
                if cb is not None:
                    try:
                        cb(body)
                    except Exception:  # noqa: BLE001 - a broken consumer must not stop the reader
                        pass
                continue
            if kind in ("done", "fail", "busy"):
                with self._lock:
                    fut, _ = self._pending.pop(key, (None, None))
                    self._streams.pop(key, None)
                    r.outstanding -= 1
                if fut is None:
                    continue
                if fut.done():  # cancelled by the caller
                    continue
                if kind == "done":
                    seq = RemoteSeq(body)
                    self.latencies_ms.append(seq.timings().get("latency_ms", 0.0))
                    fut.set_result((body["text"], seq))
                elif kind == "busy":
                    from .engine import EngineOverloaded

                    fut.set_exception(EngineOverloaded(f"replica {r.idx}: {body}"))
                else:
                    fut.set_exception(RuntimeError(f"replica {r.idx}: {body}"))
            elif kind == "stats":
                with self._lock:
                    fut, _ = self._pending.pop(key, (None, None))
                if fut is not None:
                    fut.set_result(body)
            elif kind == "closed":
                break
        with self._lock:  # replica gone: fail whatever it still owed
            lost = [(k, f) for k, (f, rr) in self._pending.items() if rr is r]
            for k, _ in lost:
                del self._pending[k]
        for _, f in lost:
            if not f.done():
                f.set_exception(RuntimeError(f"replica {r.idx} exited"))

    def stats(self, timeout_s: float = 10.0) -> dict:
        per = []
        futs = []
        for r in self.replicas:
            f: Future = Future()
            key = next(self._keys)
            with self._lock:
                self._pending[key] = (f, r)
            try:
                r.send(("stats", key, None))
            except (OSError, BrokenPipeError):
                with self._lock:
                    self._pending.pop(key, None)
                f.set_result({"healthy": False})
            futs.append((r, f))
        for r, f in futs:
            try:
                d = f.result(timeout=timeout_s)
            except Exception:  # noqa: BLE001
                d = {"healthy": False}
            d = dict(d, replica=r.idx, device=r.device, outstanding=r.outstanding)
            per.append(d)
        agg: dict = {"dp_replicas": len(self.replicas), "replicas": per,
                     "healthy": all(p.get("healthy", False) for p in per) and self._error is None}
        for k in ("requests", "finished", "prompt_tokens", "generated_tokens", "prefill_steps", "decode_steps",
                  "mixed_steps", "preemptions", "running", "waiting", "queue_depth", "rejected", "expired",
                  "cancelled", "deadline_stops"):
            agg[k] = sum(int(p.get(k, 0) or 0) for p in per)
        lat = sorted(self.latencies_ms)
        if lat:
            agg["p50_latency_ms"] = lat[len(lat) // 2]
            agg["p99_latency_ms"] = lat[min(len(lat) - 1, int(len(lat) * 0.99))]
        agg["model"] = self.engine.model_cfg.name
        return agg

    def close(self) -> None:
        for r in self.replicas:
            try:
                r.send(("close", -1, None))
            except (OSError, BrokenPipeError):
                pass
        for r in self.replicas:
            r.proc.join(timeout=60)
            if r.proc.is_alive():
                r.proc.terminate()
                r.proc.join(timeout=10)
            if r.reader is not None:
                r.reader.join(timeout=5)
            r.conn.close()


def replica_devices(n: int, first: int = 0) -> list[str]:
    """``cuda:first .. cuda:first+n-1`` (counted without initialising the GPU in this process)."""
    import torch

    have = torch.cuda.device_count()
    if have == 0:
        return ["cpu"] * n
    if first + n > have:
        raise ValueError(f"dp_replicas={n} from cuda:{first} needs {first + n} GPUs, {have} visible")
    return [f"cuda:{first + i}" for i in range(n)]
