"""UAV-aware scheduling controller (``internal/scheduler/controller.go:36-288``, S1).

Every interval: list all ``SchedulingRequest``s (scheduler.io/v1) and ``UAVMetric``s
(monitoring.io/v1); for each request whose phase is empty or Pending, validate the workload,
build candidates (UAV with a node name, battery >= minBatteryPercent when that is > 0,
collection_status empty or "active"), score = battery + 10 for a preferred node
(case-insensitive), pick the best with a stable sort and write the status through the status
subresource: ``{phase, assignedNode, assignedUAV, score, message, lastUpdated}``.

Extension: ``max_heartbeat_age_s`` (off by default, i.e. the
reference's behaviour) skips UAVs whose ``status.last_update`` is older than that.
"""
from __future__ import annotations

import logging
import threading
from typing import Optional

from ...utils.gojson import format_time_rfc3339, parse_time, utcnow
from ..cluster.backend import SCHEDULING_REQUESTS, UAV_METRICS, ClusterBackend
from ..types import SchedulingCandidate, SchedulingRequestSpec, SchedulingRequestStatus, SchedulingWorkload

log = logging.getLogger("scheduler")


def _read(m, *path):
    cur = m
    for p in path:
        if not isinstance(cur, dict):
            return None
        cur = cur.get(p)
    return cur


def read_float(m, *path) -> float:
    v = _read(m, *path)
    return float(v) if isinstance(v, (int, float)) and not isinstance(v, bool) else 0.0


def read_string(m, *path) -> str:
    v = _read(m, *path)
    return v if isinstance(v, str) else ""


class SchedulerController:
    def __init__(self, backend: ClusterBackend, interval_s: float = 10.0, max_heartbeat_age_s: float = 0.0):
        self.backend = backend
        self.interval_s = interval_s or 10.0
        self.max_heartbeat_age_s = max_heartbeat_age_s
        self._stop = threading.Event()
        self.reconciles = 0

    def run(self, stop: Optional[threading.Event] = None) -> None:
        stop = stop or self._stop
        log.info("Starting scheduler controller (interval: %ss)", self.interval_s)
        while True:
            try:
                self.reconcile()
            except Exception as e:  # noqa: BLE001
                log.error("Reconcile failed: %s", e)
            if stop.wait(self.interval_s):
                log.info("Scheduler controller stopped")
                return

    def stop(self) -> None:
        self._stop.set()

    def reconcile(self) -> int:
        """One pass; returns how many requests were decided."""
        try:
            requests = self.backend.list(SCHEDULING_REQUESTS)
        except Exception as e:  # noqa: BLE001
            raise RuntimeError(f"list scheduling requests failed: {e}") from e
        try:
            uavs = self.backend.list(UAV_METRICS)
        except Exception as e:  # noqa: BLE001
            raise RuntimeError(f"list UAV metrics failed: {e}") from e
        n = 0
        for req in requests:
            try:
                n += self.process_request(req, uavs)
            except Exception as e:  # noqa: BLE001
                md = req.get("metadata", {})
                log.error("Process request %s/%s failed: %s", md.get("namespace"), md.get("name"), e)
        self.reconciles += 1
        return n

    def process_request(self, req: dict, uavs: list) -> int:
        phase = read_string(req, "status", "phase")
        if phase and phase != "Pending":
            return 0
        spec = req.get("spec")
        if not isinstance(spec, dict):
            raise ValueError("request spec missing")
        wl = spec.get("workload") if isinstance(spec.get("workload"), dict) else {}
        rs = SchedulingRequestSpec(
            workload=SchedulingWorkload(name=wl.get("name") if isinstance(wl.get("name"), str) else "",
                                        namespace=wl.get("namespace") if isinstance(wl.get("namespace"), str) else "",
                                        type=wl.get("type") if isinstance(wl.get("type"), str) else ""),
            min_battery_percent=read_float(spec, "minBatteryPercent"),
            preferred_nodes=[s for s in spec.get("preferredNodes") or [] if isinstance(s, str)] or None)
        if not rs.workload.name or not rs.workload.namespace:
            self.update_status(req, SchedulingRequestStatus(phase="Failed", message="workload name/namespace 不能为空"))
            return 1
        cands = self.build_candidates(rs, uavs)
        if not cands:
            self.update_status(req, SchedulingRequestStatus(phase="Failed", message="无满足要求的 UAV 节点"))
            return 1
        cands.sort(key=lambda c: -c.score)  # stable, like sort.SliceStable
        c = cands[0]
        self.update_status(req, SchedulingRequestStatus(
            phase="Assigned", assigned_node=c.node_name, assigned_uav=c.uav_id, score=c.score,
            message=f"选中节点 {c.node_name} (电量 {c.battery:.1f}%)"))
        return 1

    def build_candidates(self, spec: SchedulingRequestSpec, uavs: list) -> list:
        preferred = {n.lower() for n in spec.preferred_nodes or []}
        now = utcnow()
        out = []
        for item in uavs:
            us, st = item.get("spec") or {}, item.get("status") or {}
            node = read_string(us, "node_name")
            uav_id = read_string(us, "uav_id")
            battery = read_float(us, "battery", "remaining_percent")
            cstatus = read_string(st, "collection_status").lower()
            if not node:
                continue
            if spec.min_battery_percent > 0 and battery < spec.min_battery_percent:
                continue
            if cstatus and cstatus != "active":
                continue
            hb = parse_time(read_string(st, "last_update"))
            if self.max_heartbeat_age_s > 0 and (hb is None or (now - hb).total_seconds() > self.max_heartbeat_age_s):
                continue
            score = battery + (10 if node.lower() in preferred else 0)
            out.append(SchedulingCandidate(node_name=node, uav_id=uav_id, battery=battery, last_heartbeat=hb,
                                           score=score))
        return out

    def update_status(self, req: dict, status: SchedulingRequestStatus) -> None:
        if status.last_updated is None:
            status.last_updated = utcnow()
        req["status"] = {"phase": status.phase or "Pending", "assignedNode": status.assigned_node,
                         "assignedUAV": status.assigned_uav, "score": status.score, "message": status.message,
                         "lastUpdated": format_time_rfc3339(status.last_updated)}
        self.backend.update_status(SCHEDULING_REQUESTS, req, req.get("metadata", {}).get("namespace"))
