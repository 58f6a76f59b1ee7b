"""Out-of-process HTTP load generator for the benchmarks.

The serving process (REST server threads + engine loop) shares one interpreter lock; firing 64
concurrent client requests from threads of that same process makes request arrival contend with
the server for it (the arrival of a 64-query wave spread over ~90 ms in-process).  Real clients
are remote, so ``bench.py`` runs them here, in a child process started before the parent touches
the GPU (this module imports no torch and never initialises a device).

Protocol: one JSON request per stdin line, one JSON reply per stdout line.

    {"op": "query", "port": P, "items": [[question, context], ...], "max_new_tokens": N,
     "offsets_s": [...] (optional, open-loop arrival times), "allow_errors": bool (optional),
     "slim": bool (optional: only the timing / token-count fields travel back)}
    {"op": "stage", "key": K, "items": [[question, context], ...]}   (kept for later "query"s)
    {"op": "query", "port": P, "staged": K, ...}   (the staged items: only the key crosses the pipe)
    {"op": "waves", "port": P, "staged": [K, ...], ...}   (closed-loop waves back to back, one reply)
    {"op": "podcomm", "port": P, "pairs": [[pod_a, pod_b], ...], "max_new_tokens": N}
    -> {"ok": true, "results": [...]}   (post_queries / post_pod_communication result dicts)
    -> {"ok": false, "error": "..."}
"""
from __future__ import annotations

import json
import subprocess
import sys


# what a benchmark needs from each answer: the full analysis records (answer text, prompt
# metadata) would cross the pipe twice for nothing
_SLIM = ("http_status", "http_latency_ms", "t_send_s", "error", "prompt_tokens", "completion_tokens", "ttft_ms",
         "latency_ms", "finish_reason", "type")


def serve(stdin=None, stdout=None) -> None:
    from .app import post_pod_communication, post_queries

    stdin = stdin or sys.stdin
    stdout = stdout or sys.stdout
    staged: dict = {}
    for line in stdin:
        line = line.strip()
        if not line:
            continue
        try:
            req = json.loads(line)
            if req["op"] == "stage":
                staged[str(req["key"])] = [tuple(x) for x in req["items"]]
                res = []
            elif req["op"] == "query":
                items = staged[str(req["staged"])] if req.get("staged") is not None else [tuple(x) for x in req["items"]]
                res = post_queries(req["port"], items, req["max_new_tokens"],
                                   offsets_s=req.get("offsets_s"), allow_errors=bool(req.get("allow_errors")))
                if req.get("slim"):
                    res = [{k: r[k] for k in _SLIM if k in r} for r in res]
            elif req["op"] == "waves":  # closed-loop waves back to back: wave k+1 goes out when k is answered
                res = []
                for key in req["staged"]:
                    r = post_queries(req["port"], staged[str(key)], req["max_new_tokens"],
                                     allow_errors=bool(req.get("allow_errors")))
                    res += [{k: x[k] for k in _SLIM if k in x} for x in r] if req.get("slim") else r
            elif req["op"] == "podcomm":
                res = post_pod_communication(req["port"], [tuple(x) for x in req["pairs"]], req["max_new_tokens"])
            else:
                raise ValueError(f"unknown op {req['op']!r}")
            out = {"ok": True, "results": res}
        except Exception as e:  # noqa: BLE001 - reported to the parent, which raises
            out = {"ok": False, "error": f"{type(e).__name__}: {e}"}
        stdout.write(json.dumps(out) + "\n")
        stdout.flush()


class LoadGen:
    """Parent-side handle: a persistent child running :func:`serve`.  Start it before the parent
    initialises the GPU."""

    def __init__(self, root: str | None = None):
        self.proc = subprocess.Popen([sys.executable, "-m", "k8s_llm_monitor_amd.monitor.loadgen"],
                                     stdin=subprocess.PIPE, stdout=subprocess.PIPE, text=True, bufsize=1,
                                     cwd=root)

    def _call(self, req: dict) -> list:
        self.proc.stdin.write(json.dumps(req) + "\n")
        self.proc.stdin.flush()
        line = self.proc.stdout.readline()
        if not line:
            raise RuntimeError(f"load generator exited (rc={self.proc.poll()})")
        rep = json.loads(line)
        if not rep["ok"]:
            raise RuntimeError(f"load generator: {rep['error']}")
        return rep["results"]

    def stage(self, key, items: list) -> None:
        """Hand ``items`` to the child once (outside any timed region); later post_queries(staged=key)
        send only the key."""
        self._call({"op": "stage", "key": str(key), "items": [list(x) for x in items]})

    def post_queries(self, port: int, items: list | None, max_new_tokens: int, offsets_s: list | None = None,
                     allow_errors: bool = False, slim: bool = False, staged=None) -> list:
        req = {"op": "query", "port": port, "max_new_tokens": max_new_tokens, "offsets_s": offsets_s,
               "allow_errors": allow_errors, "slim": slim}
        if staged is not None:
            req["staged"] = str(staged)
        else:
            req["items"] = [list(x) for x in items]
        return self._call(req)

    def post_waves(self, port: int, keys: list, max_new_tokens: int, allow_errors: bool = False,
                   slim: bool = False) -> list:
        """The staged waves ``keys`` as closed-loop waves inside the client process (each wave
        posted once the previous one is fully answered, as ``post_queries`` per wave) - one pipe
        round trip for all of them; returns the concatenated per-request results."""
        return self._call({"op": "waves", "port": port, "staged": [str(k) for k in keys],
                           "max_new_tokens": max_new_tokens, "allow_errors": allow_errors, "slim": slim})

    def post_pod_communication(self, port: int, pairs: list, max_new_tokens: int) -> list:
        return self._call({"op": "podcomm", "port": port, "pairs": [list(x) for x in pairs],
                           "max_new_tokens": max_new_tokens})

    def close(self) -> None:
        if self.proc.poll() is None:
            self.proc.stdin.close()
            try:
                self.proc.wait(timeout=10)
            except subprocess.TimeoutExpired:
                self.proc.kill()
                self.proc.wait()


if __name__ == "__main__":
    serve()
