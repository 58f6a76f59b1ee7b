"""MAVLink-style flight-controller simulator (``pkg/uav/mavlink_simulator.go:109-388``, U1).

Same physics and thresholds as the reference: a 10 Hz update loop; armed + AUTO flies a circle of
radius 0.001 deg at omega 0.1 rad/s around (39.9042, 116.4074), relative altitude 50 +/- 10 m;
armed discharge 0.1 %/s with the voltage / current / temperature models; battery < 20 % raises
WARNING, < 10 % CRITICAL; at most 10 health messages kept.  Differences, deliberately:

* ``get_state`` returns a deep copy (the reference shares the sensor map / message slice with the
  live state - a data race);
* ``take_off`` formats the altitude as text (the reference builds the message with
  ``string(rune(altitude))``, a garbage code point - Appendix A5 item 7);
* ``arm`` without a 3D fix returns an error message instead of silently succeeding;
* time can be driven manually (``step(dt)``) so tests are deterministic.
"""
from __future__ import annotations

import math
import random
import threading
import time
from typing import Optional

from ...utils.gojson import utcnow
from ..types import AttitudeData, BatteryData, FlightData, GPSData, HealthData, MissionData, UAVState

CENTER_LAT, CENTER_LON = 39.9042, 116.4074
UPDATE_RATE_S = 0.1


class MAVLinkSimulator:
    def __init__(self, uav_id: str, node_name: str, seed: Optional[int] = None, battery_percent: float = 100.0,
                 flight_mode: str = "STABILIZE", armed: bool = False):
        self._rng = random.Random(seed)
        now = utcnow()
        self.state = UAVState(
            uav_id=uav_id, node_name=node_name, system_time=now,
            gps=GPSData(latitude=CENTER_LAT + self._rng.random() * 0.01,
                        longitude=CENTER_LON + self._rng.random() * 0.01,
                        altitude=50.0, fix_type=3, satellite_count=12, hdop=1.0),
            attitude=AttitudeData(),
            flight=FlightData(mode=flight_mode, armed=armed, throttle_percent=0.0),
            battery=BatteryData(voltage=22.2, current=0.5, remaining_percent=battery_percent,
                                remaining_capacity=5000.0 * battery_percent / 100.0, total_capacity=5000.0,
                                temperature=25.0, cell_count=6),
            mission=MissionData(mission_state="IDLE"),
            health=HealthData(system_status="OK",
                              sensors_health={"gps": True, "compass": True, "accelerometer": True,
                                              "gyroscope": True, "barometer": True, "battery": True},
                              messages=[], last_heartbeat=now),
        )
        self._lock = threading.RLock()
        self._elapsed = 0.0
        self._thread: Optional[threading.Thread] = None
        self._stop = threading.Event()

    # ------------------------------------------------------------------ lifecycle
    def start(self) -> None:
        with self._lock:
            if self._thread is not None:
                return
            self._stop.clear()
            self._thread = threading.Thread(target=self._loop, name=f"mavlink-{self.state.uav_id}", daemon=True)
            self._thread.start()

    def stop(self) -> None:
        with self._lock:
            t = self._thread
            self._thread = None
        if t is not None:
            self._stop.set()
            t.join(timeout=2)

    def _loop(self) -> None:
        t0 = time.monotonic()
        while not self._stop.wait(UPDATE_RATE_S):
            self._update(time.monotonic() - t0)

    def step(self, dt: float = UPDATE_RATE_S) -> None:
        """Advance simulated time by ``dt`` seconds in 10 Hz ticks (test/fake-cluster driver)."""
        n = max(1, int(round(dt / UPDATE_RATE_S)))
        for _ in range(n):
            self._elapsed += UPDATE_RATE_S
            self._update(self._elapsed)

    # ------------------------------------------------------------------ commands
    def get_state(self) -> UAVState:
        with self._lock:
            return self.state.copy()

    def _msg(self, m: str) -> None:
        self.state.health.messages = (self.state.health.messages or []) + [m]

    def set_flight_mode(self, mode: str) -> None:
        with self._lock:
            self.state.flight.mode = mode
            self._msg("Flight mode changed to: " + mode)

    def arm(self) -> Optional[str]:
        with self._lock:
            if self.state.gps.fix_type < 3:
                return "GPS 3D fix required to arm"
            self.state.flight.armed = True
            self._msg("Armed")
            return None

    def disarm(self) -> None:
        with self._lock:
            self.state.flight.armed = False
            self._msg("Disarmed")

    def take_off(self, altitude: float) -> None:
        with self._lock:
            if not self.state.flight.armed:
                return
            self.state.flight.mode = "AUTO"
            self.state.mission.mission_state = "ACTIVE"
            self._msg(f"Taking off to altitude: {altitude:.1f}")

    def land(self) -> None:
        with self._lock:
            self.state.flight.mode = "LAND"
            self._msg("Landing initiated")

    def return_to_launch(self) -> None:
        with self._lock:
            self.state.flight.mode = "RTL"
            self._msg("Returning to launch")

    # ------------------------------------------------------------------ physics (updateState)
    def _update(self, t: float) -> None:
        r = self._rng
        with self._lock:
            s = self.state
            now = utcnow()
            if s.flight.armed and s.flight.mode == "AUTO":
                radius, omega = 0.001, 0.1
                s.gps.latitude = CENTER_LAT + radius * math.cos(omega * t)
                s.gps.longitude = CENTER_LON + radius * math.sin(omega * t)
                s.gps.relative_altitude = 50.0 + 10.0 * math.sin(0.05 * t)
                s.gps.ground_speed = 5.0 + r.random() * 0.5
                s.gps.course_over_ground = math.fmod(omega * t * 180 / math.pi, 360)
            s.gps.timestamp = now
            if s.flight.armed:
                s.attitude.roll = 5.0 * math.sin(0.5 * t) + r.random() * 0.5
                s.attitude.pitch = 3.0 * math.cos(0.3 * t) + r.random() * 0.3
                s.attitude.yaw = math.fmod(s.gps.course_over_ground, 360)
                s.attitude.roll_rate = r.random() * 2.0 - 1.0
                s.attitude.pitch_rate = r.random() * 2.0 - 1.0
                s.attitude.yaw_rate = r.random() * 5.0 - 2.5
            s.attitude.timestamp = now
            if s.flight.armed:
                s.flight.airspeed = s.gps.ground_speed + r.random() * 0.5
                s.flight.ground_speed = s.gps.ground_speed
                s.flight.vertical_speed = math.cos(0.05 * t) * 2.0
                s.flight.throttle_percent = 50.0 + 20.0 * math.sin(0.1 * t)
            else:
                s.flight.throttle_percent = 0.0
                s.flight.vertical_speed = 0.0
            s.flight.timestamp = now
            b = s.battery
            if s.flight.armed:
                b.remaining_percent = max(0.0, b.remaining_percent - 0.1 * UPDATE_RATE_S)
                b.remaining_capacity = b.total_capacity * b.remaining_percent / 100.0
                b.current = 10.0 + s.flight.throttle_percent * 0.2
                b.voltage = 22.2 - (100.0 - b.remaining_percent) * 0.04
                b.temperature = 25.0 + (100.0 - b.remaining_percent) * 0.3
                if b.current > 0:
                    b.time_remaining = int((b.remaining_capacity / b.current) * 3600)
            b.timestamp = now
            s.health.last_heartbeat = now
            s.health.timestamp = now
            if b.remaining_percent < 20.0 and s.health.system_status == "OK":
                s.health.system_status = "WARNING"
                s.health.warning_count += 1
                self._msg("Low battery warning")
            if b.remaining_percent < 10.0:
                s.health.system_status = "CRITICAL"
                s.health.error_count += 1
                self._msg("Critical battery level - RTL recommended")
            if len(s.health.messages or []) > 10:
                s.health.messages = s.health.messages[-10:]
            s.system_time = now
