"""UAV edge agent process (``cmd/uav-agent/main.go``, B3): MAVLink simulator + REST on ``:9090`` +
telemetry push loop to ``<master>/api/v1/uav/report``.

Flags/env as in the reference: ``-port`` (9090), ``-master-url`` / ``MASTER_URL`` (``http://``
prefixed when missing), ``-report-interval`` / ``REPORT_INTERVAL`` (Go duration, default 15s),
``NODE_NAME`` (unknown-node), ``NODE_IP`` (unknown-ip); UAV id ``UAV-<node>``.  Each report:
``UAVReport{source:"agent", status:"active", heartbeat_interval_seconds, state, metadata:{agent}}``,
HTTP timeout 15 s, 10 s per-report deadline.
"""
from __future__ import annotations

import json
import logging
import re
import threading
import time
import urllib.request
from http.server import BaseHTTPRequestHandler, ThreadingHTTPServer
from typing import Optional

from ...utils import gojson
from ...utils.gojson import utcnow
from ..types import UAVReport
from .agent_api import AgentAPI
from .simulator import MAVLinkSimulator

log = logging.getLogger("uav-agent")


def parse_go_duration(s: str) -> float:
    """time.ParseDuration subset: "1h2m3.5s", "150ms", "10s"."""
    s = s.strip()
    if not s:
        raise ValueError("empty duration")
    units = {"ns": 1e-9, "us": 1e-6, "µs": 1e-6, "ms": 1e-3, "s": 1.0, "m": 60.0, "h": 3600.0}
    total, pos = 0.0, 0
    for m in re.finditer(r"([0-9.]+)(ns|us|µs|ms|s|m|h)", s):
        if m.start() != pos:
            raise ValueError(f"time: invalid duration {s!r}")
        total += float(m.group(1)) * units[m.group(2)]
        pos = m.end()
    if pos != len(s):
        raise ValueError(f"time: invalid duration {s!r}")
    return total


class UAVAgent:
    def __init__(self, node_name: str, node_ip: str, port: int = 9090, master_url: str = "",
                 report_interval_s: float = 15.0, seed: Optional[int] = None):
        self.node_name = node_name or "unknown-node"
        self.node_ip = node_ip or "unknown-ip"
        self.uav_id = f"UAV-{self.node_name}"
        self.sim = MAVLinkSimulator(self.uav_id, self.node_name, seed=seed)
        self.api = AgentAPI(self.sim, self.uav_id, self.node_name, self.node_ip)
        self.port = port
        mu = (master_url or "").strip()
        if mu and not mu.startswith(("http://", "https://")):
            mu = "http://" + mu
        self.master_url = mu
        self.interval = report_interval_s if report_interval_s > 0 else 15.0
        self._stop = threading.Event()
        self.server: Optional[ThreadingHTTPServer] = None
        self.reports_sent = 0
        self.last_report_error = ""

    def build_report(self) -> UAVReport:
        hb = int(self.interval) or 15
        return UAVReport(node_name=self.node_name, node_ip=self.node_ip, uav_id=self.uav_id, source="agent",
                         status="active", timestamp=utcnow(), heartbeat_interval_seconds=hb,
                         state=self.sim.get_state(), metadata={"agent": "py-uav-agent"})

    def send_report(self) -> bool:
        endpoint = self.master_url.rstrip("/") + "/api/v1/uav/report"
        body = gojson.dumps(self.build_report()).encode()
        req = urllib.request.Request(endpoint, data=body, method="POST", headers={"Content-Type": "application/json"})
        try:
            with urllib.request.urlopen(req, timeout=10) as r:
                r.read()
            self.reports_sent += 1
            log.info("UAV report delivered (status %d)", r.status)
            return True
        except Exception as e:  # noqa: BLE001
            self.last_report_error = str(e)
            log.warning("Failed to send UAV report to %s: %s", endpoint, e)
            return False

    def _report_loop(self) -> None:
        self.send_report()
        while not self._stop.wait(self.interval):
            self.send_report()

    def start(self, serve_http: bool = True) -> None:
        self.sim.start()
        if serve_http:
            api = self.api

            class H(BaseHTTPRequestHandler):
                protocol_version = "HTTP/1.1"

                def log_message(self, fmt, *a):
                    log.debug(fmt, *a)

                def _do(self, method):
                    n = int(self.headers.get("Content-Length") or 0)
                    code, ctype, data = api.handle(method, self.path, self.rfile.read(n) if n else b"")
                    self.send_response(code)
                    self.send_header("Content-Type", ctype)
                    if ctype == "application/json" and self.path.split("?")[0] != "/health":
                        self.send_header("Access-Control-Allow-Origin", "*")
                    self.send_header("Content-Length", str(len(data)))
                    self.end_headers()
                    self.wfile.write(data)

                def do_GET(self):
                    self._do("GET")

                def do_POST(self):
                    self._do("POST")

            self.server = ThreadingHTTPServer(("0.0.0.0", self.port), H)
            self.server.daemon_threads = True
            threading.Thread(target=self.server.serve_forever, daemon=True, name="uav-agent-http").start()
            log.info("HTTP Server starting on port %d", self.port)
        if self.master_url:
            log.info("Telemetry reporting enabled: %s (interval %ss)", self.master_url, self.interval)
            threading.Thread(target=self._report_loop, daemon=True, name="uav-report").start()
        else:
            log.info("Master URL not configured. Telemetry reporting disabled")

    def stop(self) -> None:
        self._stop.set()
        self.sim.stop()
        if self.server is not None:
            self.server.shutdown()
