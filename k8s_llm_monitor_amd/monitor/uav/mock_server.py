#!/usr/bin/env python3
"""Stand-alone mock UAV agent (``pkg/uav/mock_server.py``, U2): stdlib HTTP on 0.0.0.0:9090
serving ``/health`` and ``/api/v1/state``, configured from env (UAV_ID, NODE_NAME, GPS_LAT/LON/ALT,
GPS_SATS, GPS_FIX, BATT_VOLTAGE/PERCENT/TEMP, FLIGHT_MODE/ARMED/SPEED).  Battery drains
``elapsed * 0.001`` floored at 20 %; ``system_status`` OK above 30 %, else WARNING.

The repository copy of the reference calls ``time.sin``/``time.cos`` (AttributeError,
Appendix A5 item 7); like the deployed ConfigMap copy, this uses ``math``.  Dependency-free so it
can be mounted into a plain ``python:3`` pod (deployments/uav-configmap.yaml).
"""
from __future__ import annotations

import json
import math
import os
import time
from datetime import datetime, timezone
from http.server import BaseHTTPRequestHandler, HTTPServer


class UAVMockSimulator:
    def __init__(self, uav_id, node_name, lat=39.9042, lon=116.4074, alt=100.0, sats=12, fix=3, voltage=22.2,
                 percent=85.0, temp=25.0, mode="AUTO", armed=True, speed=5.0):
        self.uav_id, self.node_name = uav_id, node_name
        self.lat, self.lon, self.alt, self.sats, self.fix = lat, lon, alt, sats, fix
        self.voltage, self.percent, self.temp = voltage, percent, temp
        self.mode, self.armed, self.speed = mode, armed, speed
        self.t0 = time.time()

    def state(self) -> dict:
        el = time.time() - self.t0
        pct = max(20.0, self.percent - el * 0.001)
        now = datetime.now(timezone.utc).isoformat().replace("+00:00", "Z")
        return {
            "uav_id": self.uav_id, "node_name": self.node_name, "system_time": now,
            "gps": {"latitude": self.lat + 0.0001 * math.sin(el * 0.1), "longitude": self.lon + 0.0001 * math.cos(el * 0.1),
                    "altitude": self.alt, "relative_altitude": self.alt - 50.0, "hdop": 1.0,
                    "satellite_count": self.sats, "fix_type": self.fix, "ground_speed": self.speed,
                    "course_over_ground": (el * 5) % 360, "timestamp": now},
            "attitude": {"roll": 0.0, "pitch": 0.0, "yaw": (el * 5) % 360, "roll_rate": 0.0, "pitch_rate": 0.0,
                         "yaw_rate": 0.0, "timestamp": now},
            "flight": {"mode": self.mode, "armed": self.armed, "airspeed": self.speed, "ground_speed": self.speed,
                       "vertical_speed": 0.0, "throttle_percent": 50.0 if self.armed else 0.0, "timestamp": now},
            "battery": {"voltage": self.voltage, "current": 10.0, "remaining_percent": pct,
                        "remaining_capacity": 5000.0 * pct / 100.0, "total_capacity": 5000.0,
                        "temperature": self.temp, "cell_count": 6, "time_remaining": int(5000.0 * pct / 100.0 / 10.0 * 3600),
                        "timestamp": now},
            "mission": {"current_waypoint": 0, "total_waypoints": 0, "mission_state": "ACTIVE" if self.armed else "IDLE",
                        "distance_to_wp": 0.0, "eta_to_wp": 0, "timestamp": now},
            "health": {"system_status": "OK" if pct > 30 else "WARNING",
                       "sensors_health": {"gps": True, "compass": True, "accelerometer": True, "gyroscope": True,
                                          "barometer": True, "battery": True},
                       "error_count": 0, "warning_count": 0 if pct > 30 else 1, "messages": [],
                       "last_heartbeat": now, "timestamp": now},
        }


def create_simulator_from_env() -> UAVMockSimulator:
    e = os.environ.get
    return UAVMockSimulator(
        uav_id=e("UAV_ID", "UAV-mock"), node_name=e("NODE_NAME", "unknown-node"),
        lat=float(e("GPS_LAT", "39.9042")), lon=float(e("GPS_LON", "116.4074")), alt=float(e("GPS_ALT", "100")),
        sats=int(e("GPS_SATS", "12")), fix=int(e("GPS_FIX", "3")), voltage=float(e("BATT_VOLTAGE", "22.2")),
        percent=float(e("BATT_PERCENT", "85")), temp=float(e("BATT_TEMP", "25")), mode=e("FLIGHT_MODE", "AUTO"),
        armed=e("FLIGHT_ARMED", "true").lower() == "true", speed=float(e("FLIGHT_SPEED", "5.0")))


def make_handler(sim: UAVMockSimulator):
    class UAVHandler(BaseHTTPRequestHandler):
        def log_message(self, fmt, *args):
            pass

        def _json(self, code, obj):
            data = json.dumps(obj).encode()
            self.send_response(code)
            self.send_header("Content-Type", "application/json")
            self.send_header("Access-Control-Allow-Origin", "*")
            self.send_header("Content-Length", str(len(data)))
            self.end_headers()
            self.wfile.write(data)

        def do_GET(self):
            if self.path == "/health":
                self._json(200, {"status": "healthy", "uav_id": sim.uav_id, "node_name": sim.node_name})
            elif self.path == "/api/v1/state":
                self._json(200, {"status": "success", "data": sim.state()})
            else:
                self._json(404, {"status": "error", "message": "not found"})

    return UAVHandler


def main() -> None:
    sim = create_simulator_from_env()
    port = int(os.environ.get("PORT", "9090"))
    srv = HTTPServer(("0.0.0.0", port), make_handler(sim))
    print(f"UAV mock server {sim.uav_id} on :{port}", flush=True)
    try:
        srv.serve_forever()
    except KeyboardInterrupt:
        pass


if __name__ == "__main__":
    main()
