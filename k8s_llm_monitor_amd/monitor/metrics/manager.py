"""Metrics manager (``internal/metrics/manager.go:20-565``, M1).

``collect()`` fans the enabled sources out concurrently (node, pod, network, UAV - SURVEY.md P1),
computes the cluster aggregates with the reference's health rules and swaps the snapshot under a
lock.  Reads never touch the cluster (the <10 ms metrics-read target).

Behaviour kept from the reference: pulled UAV state *replaces* the UAV map each tick
(manager.go:289-314; Appendix A5 item 2) when the pull returns anything - an empty pull no longer
wipes agent-pushed entries (that part of the quirk is fixed); agent pushes merge via
``update_uav_report``.  New: heartbeat staleness - ``get_uav_metrics`` marks an entry
``status: "stale"`` once its last heartbeat is older than 3x its heartbeat interval (SURVEY.md §5
failure detection; the reference records heartbeats but never evaluates them).
"""
from __future__ import annotations

import concurrent.futures as cf
import copy
import logging
import threading
import time
from dataclasses import dataclass
from typing import Optional

from ...utils.gojson import utcnow
from ..types import ClusterMetrics, MetricsSnapshot, NetworkMetrics, NodeMetrics, PodMetrics, UAVReport
from .sources import NetworkSource, NodeSource, PodSource, UAVSource

log = logging.getLogger("metrics")


@dataclass
class ManagerConfig:
    namespaces: list
    collect_interval_s: float = 30.0
    enable_node: bool = True
    enable_pod: bool = True
    enable_network: bool = False
    enable_custom: bool = False
    enable_uav: bool = True
    network_max_pairs: int = 5
    network_test_timeout_s: float = 10.0
    stale_after_heartbeats: float = 3.0


class MetricsManager:
    def __init__(self, backend, cfg: ManagerConfig, rtt_tester=None):
        self.cfg = cfg
        self.backend = backend
        ns = list(cfg.namespaces) or ["default"]  # the reference indexes Namespaces[0] (panics when empty)
        self.node_source = NodeSource(backend) if cfg.enable_node else None
        self.pod_source = PodSource(backend, ns) if cfg.enable_pod else None
        self.network_source = (NetworkSource(backend, rtt_tester, ns, cfg.network_max_pairs, cfg.network_test_timeout_s)
                               if cfg.enable_network and rtt_tester is not None else None)
        self.uav_source = UAVSource(backend, ns[0], "app=uav-agent", 5.0) if cfg.enable_uav else None
        now = utcnow()
        self._snapshot = MetricsSnapshot(timestamp=now, node_metrics={}, pod_metrics={}, network_metrics=[],
                                         cluster_metrics=ClusterMetrics())
        self._uav: dict = {}
        self._uav_heartbeat: dict = {}
        self._lock = threading.RLock()
        self._stop = threading.Event()
        self._thread: Optional[threading.Thread] = None
        self.collections = 0
        self.last_duration_s = 0.0
        self.listeners: list = []  # callables(snapshot) run after every collect (e.g. prompt cache refresh)

    # ------------------------------------------------------------------ lifecycle
    def start(self) -> None:
        if self._thread is not None:
            raise RuntimeError("metrics manager is already running")
        self._stop.clear()
        self._thread = threading.Thread(target=self._run, name="metrics-manager", daemon=True)
        self._thread.start()

    def _run(self) -> None:
        try:
            self.collect()
        except Exception as e:  # noqa: BLE001
            log.error("Initial metrics collection failed: %s", e)
        while not self._stop.wait(self.cfg.collect_interval_s):
            try:
                self.collect()
            except Exception as e:  # noqa: BLE001
                log.error("Failed to collect metrics: %s", e)

    def stop(self) -> None:
        if self._thread is None:
            raise RuntimeError("metrics manager is not running")
        self._stop.set()
        self._thread.join(timeout=5)
        self._thread = None

    @property
    def running(self) -> bool:
        return self._thread is not None

    # ------------------------------------------------------------------ collect
    def collect(self) -> MetricsSnapshot:
        t0 = time.perf_counter()
        start = utcnow()
        snap = MetricsSnapshot(timestamp=start, node_metrics={}, pod_metrics={}, network_metrics=[],
                               cluster_metrics=ClusterMetrics(timestamp=start))
        errors: dict = {}
        uav_pulled: Optional[dict] = None
        jobs = {}
        with cf.ThreadPoolExecutor(max_workers=4) as ex:
            if self.node_source:
                jobs["node"] = ex.submit(self.node_source.collect)
            if self.pod_source:
                jobs["pod"] = ex.submit(self.pod_source.collect)
            if self.network_source:
                jobs["network"] = ex.submit(self.network_source.collect)
            if self.uav_source:
                jobs["uav"] = ex.submit(self.uav_source.collect)
            for k, f in jobs.items():
                try:
                    r = f.result()
                except Exception as e:  # noqa: BLE001 - per-source isolation (manager.go:321-333)
                    errors[k] = e
                    log.error("Failed to collect %s metrics: %s", k, e)
                    continue
                if k == "node":
                    snap.node_metrics = r
                elif k == "pod":
                    snap.pod_metrics = r
                elif k == "network":
                    snap.network_metrics = r
                else:
                    now = utcnow()
                    uav_pulled = {n: {"node_name": n, "status": "active", "source": "pull", "timestamp": now,
                                      "last_heartbeat": now, "state": s} for n, s in r.items()}
        calculate_cluster_metrics(snap)
        with self._lock:
            self._snapshot = snap
            if uav_pulled:
                self._uav = uav_pulled
                for n, e in uav_pulled.items():
                    self._uav_heartbeat[n] = e["last_heartbeat"]
            self.collections += 1
        self.last_duration_s = time.perf_counter() - t0
        log.info("Metrics collection completed in %.3fs (nodes: %d, pods: %d, network: %d, uavs: %d)",
                 self.last_duration_s, len(snap.node_metrics), len(snap.pod_metrics), len(snap.network_metrics),
                 len(uav_pulled or {}))
        for cb in list(self.listeners):
            try:
                cb(snap)
            except Exception as e:  # noqa: BLE001
                log.warning("snapshot listener failed: %s", e)
        if "node" in errors:
            raise errors["node"]
        if "pod" in errors:
            raise errors["pod"]
        return snap

    # ------------------------------------------------------------------ reads
    def get_latest_snapshot(self) -> MetricsSnapshot:
        with self._lock:
            return self._snapshot

    def get_node_metrics(self, name: str) -> NodeMetrics:
        with self._lock:
            m = (self._snapshot.node_metrics or {}).get(name)
        if m is None:
            raise KeyError(f"metrics not found for node: {name}")
        return m

    def get_pod_metrics(self, namespace: str, name: str) -> PodMetrics:
        with self._lock:
            m = (self._snapshot.pod_metrics or {}).get(f"{namespace}/{name}")
        if m is None:
            raise KeyError(f"metrics not found for pod: {namespace}/{name}")
        return m

    def get_cluster_metrics(self) -> ClusterMetrics:
        with self._lock:
            return self._snapshot.cluster_metrics

    def get_network_metrics(self) -> list:
        with self._lock:
            return self._snapshot.network_metrics

    def test_pod_communication(self, source: str, target: str) -> NetworkMetrics:
        if self.network_source is None:
            raise RuntimeError("network metrics collector not enabled")
        return self.network_source.test_pod_connectivity(source, target)

    # ------------------------------------------------------------------ UAV push / read
    def update_uav_report(self, r: UAVReport) -> None:
        if r is None or not r.node_name:
            return
        ts = r.timestamp or utcnow()
        entry = {"node_name": r.node_name, "uav_id": r.uav_id, "status": r.status or "active",
                 "source": r.source or "agent", "timestamp": ts, "last_heartbeat": ts}
        if r.node_ip:
            entry["node_ip"] = r.node_ip
        if r.heartbeat_interval_seconds > 0:
            entry["heartbeat_interval_seconds"] = r.heartbeat_interval_seconds
        if r.metadata:
            entry["metadata"] = dict(r.metadata)
        if r.state is not None:
            entry["state"] = r.state.copy()
        with self._lock:
            self._uav[r.node_name] = entry
            self._uav_heartbeat[r.node_name] = ts

    def _with_staleness(self, entry: dict, now) -> dict:
        e = dict(entry)
        hb = e.get("last_heartbeat")
        interval = e.get("heartbeat_interval_seconds") or self.cfg.collect_interval_s
        if hb is not None and (now - hb).total_seconds() > self.cfg.stale_after_heartbeats * interval:
            e["status"] = "stale"
        return e

    def get_uav_metrics(self) -> dict:
        now = utcnow()
        with self._lock:
            return {k: self._with_staleness(v, now) for k, v in self._uav.items()}

    def get_single_uav_metrics(self, node: str) -> Optional[dict]:
        with self._lock:
            e = self._uav.get(node)
        return None if e is None else self._with_staleness(e, utcnow())


def calculate_cluster_metrics(snap: MetricsSnapshot) -> None:
    """manager.go:493-565: totals, usage rates, issues, healthy|warning|critical."""
    c = snap.cluster_metrics
    nodes = snap.node_metrics or {}
    pods = snap.pod_metrics or {}
    c.total_nodes = len(nodes)
    c.healthy_nodes = sum(1 for n in nodes.values() if n.healthy)
    c.total_pods = len(pods)
    c.running_pods = sum(1 for p in pods.values() if p.phase == "Running")
    c.total_cpu = sum(n.cpu_capacity for n in nodes.values())
    c.used_cpu = sum(n.cpu_usage for n in nodes.values())
    c.total_memory = sum(n.memory_capacity for n in nodes.values())
    c.used_memory = sum(n.memory_usage for n in nodes.values())
    c.total_gpus = sum(n.gpu_count for n in nodes.values())
    c.available_gpus = sum(1 for n in nodes.values() for u in (n.gpu_usage or []) if u < 50.0)
    c.cpu_usage_rate = c.used_cpu / c.total_cpu * 100.0 if c.total_cpu > 0 else 0.0
    c.memory_usage_rate = c.used_memory / c.total_memory * 100.0 if c.total_memory > 0 else 0.0
    issues = []
    if c.healthy_nodes < c.total_nodes:
        issues.append(f"{c.total_nodes - c.healthy_nodes} nodes are unhealthy")
    if c.cpu_usage_rate > 80:
        issues.append(f"High CPU usage: {c.cpu_usage_rate:.1f}%")
    if c.memory_usage_rate > 80:
        issues.append(f"High memory usage: {c.memory_usage_rate:.1f}%")
    c.issues = issues
    if not issues:
        c.health_status = "healthy"
    elif c.cpu_usage_rate > 90 or c.memory_usage_rate > 90 or c.healthy_nodes < c.total_nodes // 2:
        c.health_status = "critical"
    else:
        c.health_status = "warning"
