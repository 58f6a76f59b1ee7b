"""Kubernetes REST backend on the Python standard library (no client-go / kubernetes package
offline; SURVEY.md §7.1 "K8s API via a tiny stdlib REST client").

* auth: kubeconfig (``k8s.kubeconfig`` or ``$KUBECONFIG`` / ``~/.kube/config``: server, CA, bearer
  token, client certificate, ``exec`` credential plugins, insecure-skip-tls-verify) or the
  in-cluster service account (``rest.InClusterConfig`` semantics);
* typed + dynamic access by GVR: list / get / create / update / update_status / delete;
* watch: chunked JSON-lines stream (``?watch=1``) with resourceVersion resume;
* exec: the ``v4.channel.k8s.io`` WebSocket protocol (instead of SPDY, which client-go uses in
  ``rtt_tester.go:184-215``) with a minimal RFC 6455 client;
* pod logs; plain HTTP to in-cluster endpoints (UAV agents).
"""
from __future__ import annotations

import base64
import http.client
import json
import os
import socket
import ssl
import struct
import subprocess
import tempfile
import time
from typing import Iterator, Optional
from urllib.parse import quote, urlencode, urlparse

import yaml

from .backend import GVR, KINDS, ApiError, ClusterBackend, ExecError

SA_DIR = "/var/run/secrets/kubernetes.io/serviceaccount"


class KubeConfigError(Exception):
    pass


class KubeRESTBackend(ClusterBackend):
    def __init__(self, server: str, token: str = "", ca_file: Optional[str] = None, cert_file: Optional[str] = None,
                 key_file: Optional[str] = None, insecure: bool = False, timeout_s: float = 30.0,
                 token_refresher=None):
        u = urlparse(server)
        self.scheme = u.scheme or "https"
        self.host = u.hostname or "127.0.0.1"
        self.port = u.port or (443 if self.scheme == "https" else 80)
        self.base_path = u.path.rstrip("/")
        self.token = token
        self.timeout = timeout_s
        self._refresh = token_refresher
        self.ctx = None
        if self.scheme == "https":
            self.ctx = ssl.create_default_context(cafile=ca_file) if ca_file else ssl.create_default_context()
            if insecure:
                self.ctx.check_hostname = False
                self.ctx.verify_mode = ssl.CERT_NONE
            if cert_file:
                self.ctx.load_cert_chain(cert_file, key_file)

    # ------------------------------------------------------------------ construction
    @classmethod
    def in_cluster(cls) -> "KubeRESTBackend":
        host, port = os.environ.get("KUBERNETES_SERVICE_HOST"), os.environ.get("KUBERNETES_SERVICE_PORT")
        tok = os.path.join(SA_DIR, "token")
        if not host or not port or not os.path.exists(tok):
            raise KubeConfigError("unable to load in-cluster configuration, KUBERNETES_SERVICE_HOST and "
                                  "KUBERNETES_SERVICE_PORT must be defined")
        with open(tok) as fh:
            token = fh.read().strip()
        h = f"[{host}]" if ":" in host else host
        return cls(f"https://{h}:{port}", token=token, ca_file=os.path.join(SA_DIR, "ca.crt"),
                   token_refresher=lambda: open(tok).read().strip())

    @classmethod
    def from_kubeconfig(cls, path: str, context: Optional[str] = None) -> "KubeRESTBackend":
        try:
            with open(os.path.expanduser(path)) as fh:
                kc = yaml.safe_load(fh) or {}
        except OSError as e:
            raise KubeConfigError(f"stat {path}: no such file or directory") from e
        ctx_name = context or kc.get("current-context")
        ctxs = {c["name"]: c.get("context", {}) for c in kc.get("contexts") or []}
        if ctx_name not in ctxs:
            raise KubeConfigError(f'context "{ctx_name}" does not exist')
        cx = ctxs[ctx_name]
        clusters = {c["name"]: c.get("cluster", {}) for c in kc.get("clusters") or []}
        users = {u["name"]: u.get("user", {}) for u in kc.get("users") or []}
        cl, us = clusters.get(cx.get("cluster"), {}), users.get(cx.get("user"), {})
        base = os.path.dirname(os.path.abspath(os.path.expanduser(path)))

        def materialise(data_key: str, file_key: str, src: dict) -> Optional[str]:
            if src.get(data_key):
                f = tempfile.NamedTemporaryFile(delete=False, suffix=".pem")
                f.write(base64.b64decode(src[data_key]))
                f.close()
                return f.name
            if src.get(file_key):
                p = src[file_key]
                return p if os.path.isabs(p) else os.path.join(base, p)
            return None

        token = us.get("token", "")
        if not token and us.get("tokenFile"):
            with open(us["tokenFile"]) as fh:
                token = fh.read().strip()
        refresher = None
        if us.get("exec"):
            refresher = _exec_plugin(us["exec"])
            token = refresher()
        return cls(cl.get("server", ""), token=token,
                   ca_file=materialise("certificate-authority-data", "certificate-authority", cl),
                   cert_file=materialise("client-certificate-data", "client-certificate", us),
                   key_file=materialise("client-key-data", "client-key", us),
                   insecure=bool(cl.get("insecure-skip-tls-verify")), token_refresher=refresher)

    @classmethod
    def from_config(cls, kubeconfig: str = "") -> "KubeRESTBackend":
        """``k8s.kubeconfig`` if set, else in-cluster, else $KUBECONFIG / ~/.kube/config
        (client.go:35-77 + clientcmd fallback)."""
        if kubeconfig:
            return cls.from_kubeconfig(kubeconfig)
        try:
            return cls.in_cluster()
        except KubeConfigError:
            for p in (os.environ.get("KUBECONFIG", "").split(os.pathsep)[0], "~/.kube/config"):
                if p and os.path.exists(os.path.expanduser(p)):
                    return cls.from_kubeconfig(p)
            raise

    # ------------------------------------------------------------------ HTTP plumbing
    def _conn(self, timeout: Optional[float] = None):
        t = timeout or self.timeout
        if self.scheme == "https":
            return http.client.HTTPSConnection(self.host, self.port, timeout=t, context=self.ctx)
        return http.client.HTTPConnection(self.host, self.port, timeout=t)

    def _headers(self, extra: Optional[dict] = None) -> dict:
        h = {"Accept": "application/json", "User-Agent": "k8s-llm-monitor-amd/1.0"}
        if self.token:
            h["Authorization"] = f"Bearer {self.token}"
        h.update(extra or {})
        return h

    def _path(self, gvr: GVR, namespace: Optional[str] = None, name: str = "", sub: str = "") -> str:
        root = f"/api/{gvr.version}" if not gvr.group else f"/apis/{gvr.group}/{gvr.version}"
        p = self.base_path + root
        if gvr.namespaced and namespace:
            p += f"/namespaces/{quote(namespace)}"
        p += f"/{gvr.resource}"
        if name:
            p += f"/{quote(name)}"
        if sub:
            p += f"/{sub}"
        return p

    def _request(self, method: str, path: str, body=None, query: Optional[dict] = None, retry: bool = True):
        url = path + (("?" + urlencode(query, doseq=True)) if query else "")
        data = json.dumps(body).encode() if body is not None else None
        conn = self._conn()
        try:
            conn.request(method, url, data, self._headers({"Content-Type": "application/json"} if data else None))
            r = conn.getresponse()
            raw = r.read()
        finally:
            conn.close()
        if r.status == 401 and retry and self._refresh is not None:
            self.token = self._refresh()
            return self._request(method, path, body, query, retry=False)
        if r.status >= 400:
            try:
                st = json.loads(raw)
                raise ApiError(r.status, st.get("reason", ""), st.get("message", raw.decode(errors="replace")))
            except ValueError:
                raise ApiError(r.status, "", raw.decode(errors="replace")) from None
        return json.loads(raw) if raw else {}

    # ------------------------------------------------------------------ ClusterBackend
    def server_version(self) -> dict:
        return self._request("GET", self.base_path + "/version")

    def list(self, gvr: GVR, namespace: Optional[str] = None, label_selector: str = "", field_selector: str = "",
             limit: int = 0) -> list[dict]:
        q = {}
        if label_selector:
            q["labelSelector"] = label_selector
        if field_selector:
            q["fieldSelector"] = field_selector
        if limit:
            q["limit"] = str(limit)
        d = self._request("GET", self._path(gvr, namespace), query=q)
        items = d.get("items") or []
        kind = (d.get("kind") or "").removesuffix("List")
        if kind in ("", "Table"):
            kind = KINDS.get(gvr, "")
        for it in items:  # list items carry no apiVersion/kind; restore them like the dynamic client
            it.setdefault("apiVersion", gvr.api_version)
            if kind:
                it.setdefault("kind", kind)
        return items

    def get(self, gvr: GVR, name: str, namespace: Optional[str] = None) -> dict:
        return self._request("GET", self._path(gvr, namespace, name))

    def create(self, gvr: GVR, obj: dict, namespace: Optional[str] = None) -> dict:
        return self._request("POST", self._path(gvr, namespace or obj.get("metadata", {}).get("namespace")), obj)

    def update(self, gvr: GVR, obj: dict, namespace: Optional[str] = None) -> dict:
        md = obj.get("metadata", {})
        return self._request("PUT", self._path(gvr, namespace or md.get("namespace"), md.get("name", "")), obj)

    def update_status(self, gvr: GVR, obj: dict, namespace: Optional[str] = None) -> dict:
        md = obj.get("metadata", {})
        return self._request("PUT", self._path(gvr, namespace or md.get("namespace"), md.get("name", ""), "status"),
                             obj)

    def delete(self, gvr: GVR, name: str, namespace: Optional[str] = None) -> None:
        self._request("DELETE", self._path(gvr, namespace, name))

    def watch(self, gvr: GVR, namespace: Optional[str] = None, resource_version: str = "", timeout_s: float = 300.0,
              stop=None) -> Iterator[tuple[str, dict]]:
        q = {"watch": "1", "timeoutSeconds": str(int(timeout_s)), "allowWatchBookmarks": "true"}
        if resource_version:
            q["resourceVersion"] = resource_version
        conn = self._conn(timeout=timeout_s + 10)
        try:
            conn.request("GET", self._path(gvr, namespace) + "?" + urlencode(q), headers=self._headers())
            r = conn.getresponse()
            if r.status >= 400:
                raise ApiError(r.status, "", r.read().decode(errors="replace"))
            buf = b""
            while stop is None or not stop.is_set():
                chunk = r.read1(65536) if hasattr(r, "read1") else r.read(4096)
                if not chunk:
                    return
                buf += chunk
                while b"\n" in buf:
                    line, buf = buf.split(b"\n", 1)
                    if line.strip():
                        ev = json.loads(line)
                        yield ev.get("type", ""), ev.get("object") or {}
        finally:
            conn.close()

    def pod_logs(self, namespace: str, pod: str, tail_lines: int = 100) -> str:
        conn = self._conn()
        try:
            conn.request("GET", self._path(GVR("", "v1", "pods"), namespace, pod, "log") + f"?tailLines={tail_lines}",
                         headers=self._headers({"Accept": "*/*"}))
            r = conn.getresponse()
            data = r.read()
        finally:
            conn.close()
        if r.status >= 400:
            raise ApiError(r.status, "", data.decode(errors="replace"))
        return data.decode(errors="replace")

    def exec(self, namespace: str, pod: str, container: str, command: list[str],
             timeout_s: float = 30.0) -> tuple[str, str]:
        q = [("container", container)] + [("command", c) for c in command] + [("stdout", "true"), ("stderr", "true")]
        path = self._path(GVR("", "v1", "pods"), namespace, pod, "exec") + "?" + urlencode(q)
        ws = _WebSocket.connect(self, path, "v4.channel.k8s.io", timeout_s)
        out, err, status = [], [], None
        try:
            deadline = time.monotonic() + timeout_s
            while time.monotonic() < deadline:
                msg = ws.recv(max(0.1, deadline - time.monotonic()))
                if msg is None:
                    break
                if not msg:
                    continue
                ch, payload = msg[0], msg[1:]
                if ch == 1:
                    out.append(payload)
                elif ch == 2:
                    err.append(payload)
                elif ch == 3:
                    status = json.loads(payload or b"{}")
            else:
                raise ExecError("command execution timed out")
        finally:
            ws.close()
        so, se = b"".join(out).decode(errors="replace"), b"".join(err).decode(errors="replace")
        if status and status.get("status") == "Failure":
            raise ExecError(f"{status.get('message', 'command failed')}, stderr: {se}")
        return so, se

    def http_request(self, method: str, url: str, body: Optional[bytes] = None,
                     timeout_s: float = 5.0) -> tuple[int, bytes]:
        u = urlparse(url)
        conn = http.client.HTTPConnection(u.hostname, u.port or 80, timeout=timeout_s)
        try:
            conn.request(method, u.path + (("?" + u.query) if u.query else ""), body,
                         {"Content-Type": "application/json"} if body else {})
            r = conn.getresponse()
            return r.status, r.read()
        finally:
            conn.close()


def _exec_plugin(spec: dict):
    """client.authentication.k8s.io ExecCredential plugins (aws/gke/oidc helpers)."""
    def run() -> str:
        env = dict(os.environ)
        for e in spec.get("env") or []:
            env[e["name"]] = e["value"]
        out = subprocess.run([spec["command"]] + list(spec.get("args") or []), capture_output=True, env=env,
                             timeout=60, check=True).stdout
        return json.loads(out)["status"]["token"]
    return run


class _WebSocket:
    """Just enough RFC 6455 for the exec channel protocol (client side, binary frames)."""

    def __init__(self, sock):
        self.sock = sock
        self.buf = b""

    @classmethod
    def connect(cls, be: KubeRESTBackend, path: str, protocol: str, timeout_s: float) -> "_WebSocket":
        raw = socket.create_connection((be.host, be.port), timeout=timeout_s)
        sock = be.ctx.wrap_socket(raw, server_hostname=be.host) if be.scheme == "https" else raw
        key = base64.b64encode(os.urandom(16)).decode()
        hdr = [f"GET {path} HTTP/1.1", f"Host: {be.host}:{be.port}", "Upgrade: websocket", "Connection: Upgrade",
               f"Sec-WebSocket-Key: {key}", "Sec-WebSocket-Version: 13", f"Sec-WebSocket-Protocol: {protocol}"]
        if be.token:
            hdr.append(f"Authorization: Bearer {be.token}")
        sock.sendall(("\r\n".join(hdr) + "\r\n\r\n").encode())
        ws = cls(sock)
        head = ws._read_until(b"\r\n\r\n")
        status = head.split(b"\r\n", 1)[0]
        if b" 101 " not in status + b" ":
            raise ExecError(f"unable to upgrade connection: {status.decode(errors='replace')}")
        return ws

    def _read_until(self, marker: bytes) -> bytes:
        while marker not in self.buf:
            d = self.sock.recv(65536)
            if not d:
                raise ExecError("connection closed during handshake")
            self.buf += d
        head, self.buf = self.buf.split(marker, 1)
        return head

    def _read(self, n: int) -> bytes:
        while len(self.buf) < n:
            d = self.sock.recv(65536)
            if not d:
                raise EOFError
            self.buf += d
        out, self.buf = self.buf[:n], self.buf[n:]
        return out

    def recv(self, timeout: float) -> Optional[bytes]:
        self.sock.settimeout(timeout)
        try:
            b0, b1 = self._read(2)
            op, ln = b0 & 0x0F, b1 & 0x7F
            if ln == 126:
                ln = struct.unpack(">H", self._read(2))[0]
            elif ln == 127:
                ln = struct.unpack(">Q", self._read(8))[0]
            mask = self._read(4) if b1 & 0x80 else None
            data = self._read(ln)
            if mask:
                data = bytes(c ^ mask[i % 4] for i, c in enumerate(data))
        except (EOFError, socket.timeout, OSError):
            return None
        if op == 8:  # close
            return None
        if op == 9:  # ping -> pong
            self._send(10, data)
            return b""
        return data

    def _send(self, op: int, data: bytes) -> None:
        m = os.urandom(4)
        hdr = bytes([0x80 | op])
        n = len(data)
        if n < 126:
            hdr += bytes([0x80 | n])
        elif n < 65536:
            hdr += bytes([0x80 | 126]) + struct.pack(">H", n)
        else:
            hdr += bytes([0x80 | 127]) + struct.pack(">Q", n)
        self.sock.sendall(hdr + m + bytes(c ^ m[i % 4] for i, c in enumerate(data)))

    def close(self) -> None:
        try:
            self._send(8, b"")
        except OSError:
            pass
        try:
            self.sock.close()
        except OSError:
            pass
