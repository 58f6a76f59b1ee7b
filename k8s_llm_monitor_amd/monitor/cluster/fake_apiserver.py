"""Serve a :class:`FakeCluster` over the real Kubernetes REST paths, so the stdlib
:class:`KubeRESTBackend` (URL building, auth header, list/get/create/update/status, watch streaming,
errors as ``Status`` objects) can be exercised end to end without a cluster - including by the
``server`` process itself (``kubeconfig`` pointing at this endpoint).

    python -m k8s_llm_monitor_amd.monitor.cluster.fake_apiserver --port 6443
"""
from __future__ import annotations

import argparse
import json
import re
import threading
from http.server import BaseHTTPRequestHandler, ThreadingHTTPServer
from urllib.parse import parse_qs, urlparse

from .backend import GVR, KINDS, ApiError
from .fake import FakeCluster

_PATH = re.compile(r"^/(?:api/(?P<cv>v1)|apis/(?P<g>[^/]+)/(?P<v>[^/]+))"
                   r"(?:/namespaces/(?P<ns>[^/]+))?/(?P<res>[^/]+)(?:/(?P<name>[^/]+))?(?:/(?P<sub>[^/]+))?$")
CLUSTER_SCOPED = {"nodes", "namespaces", "customresourcedefinitions"}


def make_handler(fc: FakeCluster, token: str = ""):
    class H(BaseHTTPRequestHandler):
        protocol_version = "HTTP/1.1"

        def log_message(self, *a):
            pass

        def _send(self, code: int, obj, chunked: bool = False):
            data = json.dumps(obj).encode()
            self.send_response(code)
            self.send_header("Content-Type", "application/json")
            self.send_header("Content-Length", str(len(data)))
            self.end_headers()
            self.wfile.write(data)

        def _status(self, e: ApiError):
            self._send(e.code, {"kind": "Status", "apiVersion": "v1", "status": "Failure", "message": e.message,
                                "reason": e.reason, "code": e.code})

        def _route(self, method: str):
            if token and self.headers.get("Authorization") != f"Bearer {token}":
                return self._status(ApiError(401, "Unauthorized", "Unauthorized"))
            u = urlparse(self.path)
            q = {k: v[0] for k, v in parse_qs(u.query).items()}
            if u.path == "/version":
                return self._send(200, fc.server_version())
            m = _PATH.match(u.path)
            if not m:
                return self._status(ApiError(404, "NotFound", "the server could not find the requested resource"))
            res = m["res"]
            gvr = GVR(m["g"] or "", m["v"] or m["cv"], res, res not in CLUSTER_SCOPED)
            ns, name, sub = m["ns"], m["name"], m["sub"]
            n = int(self.headers.get("Content-Length") or 0)
            body = json.loads(self.rfile.read(n)) if n else None
            try:
                if method == "GET" and name and sub == "log":
                    data = fc.pod_logs(ns, name, int(q.get("tailLines", 100))).encode()
                    self.send_response(200)
                    self.send_header("Content-Type", "text/plain")
                    self.send_header("Content-Length", str(len(data)))
                    self.end_headers()
                    self.wfile.write(data)
                    return
                if method == "GET" and not name and q.get("watch") in ("1", "true"):
                    return self._watch(gvr, ns, q)
                if method == "GET" and not name:
                    items = fc.list(gvr, ns, q.get("labelSelector", ""), q.get("fieldSelector", ""),
                                    int(q.get("limit", 0)))
                    for it in items:  # the API server omits these on list items
                        it.pop("apiVersion", None)
                        it.pop("kind", None)
                    return self._send(200, {"kind": KINDS.get(gvr, "Object") + "List", "apiVersion": gvr.api_version, "items": items,
                                            "metadata": {"resourceVersion": str(len(fc._log))}})
                if method == "GET":
                    return self._send(200, fc.get(gvr, name, ns))
                if method == "POST":
                    return self._send(201, fc.create(gvr, body, ns))
                if method == "PUT" and sub == "status":
                    return self._send(200, fc.update_status(gvr, body, ns))
                if method == "PUT":
                    return self._send(200, fc.update(gvr, body, ns))
                if method == "DELETE":
                    fc.delete(gvr, name, ns)
                    return self._send(200, {"kind": "Status", "status": "Success"})
            except ApiError as e:
                return self._status(e)
            return self._status(ApiError(405, "MethodNotAllowed", "method not allowed"))

        def _watch(self, gvr, ns, q):
            self.send_response(200)
            self.send_header("Content-Type", "application/json")
            self.send_header("Transfer-Encoding", "chunked")
            self.end_headers()
            try:
                for etype, obj in fc.watch(gvr, ns, q.get("resourceVersion", ""), float(q.get("timeoutSeconds", 30))):
                    line = json.dumps({"type": etype, "object": obj}).encode() + b"\n"
                    self.wfile.write(f"{len(line):x}\r\n".encode() + line + b"\r\n")
                    self.wfile.flush()
                self.wfile.write(b"0\r\n\r\n")
            except (BrokenPipeError, ConnectionResetError):
                pass

        def do_GET(self):
            self._route("GET")

        def do_POST(self):
            self._route("POST")

        def do_PUT(self):
            self._route("PUT")

        def do_DELETE(self):
            self._route("DELETE")

    return H


def serve(fc: FakeCluster, host: str = "127.0.0.1", port: int = 0, token: str = ""):
    srv = ThreadingHTTPServer((host, port), make_handler(fc, token))
    srv.daemon_threads = True
    threading.Thread(target=srv.serve_forever, daemon=True, name="fake-apiserver").start()
    return srv


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--port", type=int, default=6443)
    ap.add_argument("--nodes", type=int, default=3)
    ap.add_argument("--token", default="")
    a = ap.parse_args()
    srv = serve(FakeCluster.build(n_nodes=a.nodes), "127.0.0.1", a.port, a.token)
    print(f"fake kube-apiserver on http://127.0.0.1:{srv.server_address[1]}", flush=True)
    threading.Event().wait()


if __name__ == "__main__":
    main()
