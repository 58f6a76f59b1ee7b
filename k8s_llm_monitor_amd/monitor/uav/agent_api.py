"""The UAV edge agent's REST surface (``cmd/uav-agent/main.go:84-280``)
as a transport-independent router: ``handle(method, path, body) -> (status, content_type, bytes)``.
The real agent serves it over HTTP (``agent.py``); the FakeCluster routes in-cluster requests to
``http://<podIP>:9090`` through the same function, so the metrics collector exercises identical
responses in tests and benchmarks.
"""
from __future__ import annotations

import json
from typing import Optional

from ...utils import gojson
from ...utils.gojson import utcnow
from .simulator import MAVLinkSimulator

TEXT = "text/plain; charset=utf-8"
JSON = "application/json"


def _err(code: int, msg: str) -> tuple[int, str, bytes]:
    return code, TEXT, (msg + "\n").encode()


class AgentAPI:
    def __init__(self, sim: MAVLinkSimulator, uav_id: str, node_name: str, node_ip: str):
        self.sim, self.uav_id, self.node_name, self.node_ip = sim, uav_id, node_name, node_ip

    def handle(self, method: str, path: str, body: Optional[bytes] = None) -> tuple[int, str, bytes]:
        path = path.split("?", 1)[0]
        ok = lambda d: (200, JSON, gojson.encode(d))  # noqa: E731
        if path == "/health":
            return ok({"status": "healthy", "uav_id": self.uav_id, "node_name": self.node_name,
                       "node_ip": self.node_ip, "timestamp": utcnow()})
        if path == "/api/v1/state":
            if method != "GET":
                return _err(405, "Method not allowed")
            return ok({"status": "success", "data": self.sim.get_state()})
        sub = {"/api/v1/gps": "gps", "/api/v1/attitude": "attitude", "/api/v1/battery": "battery",
               "/api/v1/flight": "flight"}.get(path)
        if sub:  # any method, like the reference
            return ok({"status": "success", "data": getattr(self.sim.get_state(), sub)})
        if path.startswith("/api/v1/command/"):
            if method != "POST":
                return _err(405, "Method not allowed")
            cmd = path[len("/api/v1/command/"):]
            if cmd == "arm":
                err = self.sim.arm()
                if err:
                    return ok({"status": "error", "message": err})
                return ok({"status": "success", "message": "Armed successfully"})
            if cmd == "disarm":
                self.sim.disarm()
                return ok({"status": "success", "message": "Disarmed successfully"})
            if cmd in ("takeoff", "mode"):
                try:
                    req = json.loads(body or b"")
                    if not isinstance(req, dict):
                        raise ValueError
                except ValueError:
                    return _err(400, "Invalid request body")
                if cmd == "takeoff":
                    alt = float(req.get("altitude") or 0.0) or 50.0
                    self.sim.take_off(alt)
                    return ok({"status": "success", "message": f"Taking off to {alt:.1f}m"})
                mode = str(req.get("mode") or "")
                self.sim.set_flight_mode(mode)
                return ok({"status": "success", "message": f"Flight mode set to {mode}"})
            if cmd == "land":
                self.sim.land()
                return ok({"status": "success", "message": "Landing initiated"})
            if cmd == "rtl":
                self.sim.return_to_launch()
                return ok({"status": "success", "message": "Returning to launch"})
        return _err(404, "404 page not found")
