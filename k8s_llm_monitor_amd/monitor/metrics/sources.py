"""Metrics sources (``internal/metrics/sources/*.go``, M2-M5) over a :class:`ClusterBackend`.

* NodeSource    - nodes + metrics.k8s.io NodeMetrics; degrades to zero usage when metrics-server
                  is unavailable (node_metrics.go:37-70); health = Ready and no Memory/Disk/PID
                  pressure or NetworkUnavailable (:95-205).
* PodSource     - per namespace (``""`` = all), requests/limits/usage, rates relative to the
                  *limit* (pod_metrics.go:101-218).
* NetworkSource - Running pods with IPs, cross-node pairs first, capped at ``max_pairs``, tested
                  with a concurrency limit of 3 (network_metrics.go:66-206) via the RTT tester.
* UAVSource     - Running ``app=uav-agent`` pods, one concurrent GET ``:9090/api/v1/state`` each
                  (uav_metrics.go:62-172).
"""
from __future__ import annotations

import json
import logging
import concurrent.futures as cf
from dataclasses import dataclass
from typing import Optional

from ...utils.gojson import ZERO_TIME, parse_time, utcnow
from ..cluster.backend import NODE_METRICS, NODES, POD_METRICS, PODS, ApiError, ClusterBackend, milli_value, value
from ..types import ContainerMetrics, NetworkMetrics, NodeMetrics, PodMetrics, UAVState

log = logging.getLogger("metrics")


def _q(d: Optional[dict], key: str, milli: bool) -> Optional[int]:
    if not d or key not in d:
        return None
    return milli_value(d[key]) if milli else value(d[key])


class NodeSource:
    def __init__(self, backend: ClusterBackend):
        self.backend = backend

    def collect(self) -> dict:
        nodes = self.backend.list(NODES)
        try:
            nm = {m["metadata"]["name"]: m for m in self.backend.list(NODE_METRICS)}
        except (ApiError, OSError) as e:
            log.warning("Failed to get node metrics from metrics server: %s (metrics may be incomplete)", e)
            nm = {}
        return {n["metadata"]["name"]: build_node_metrics(n, nm.get(n["metadata"]["name"])) for n in nodes}

    def collect_single(self, name: str) -> NodeMetrics:
        node = self.backend.get(NODES, name)
        try:
            m = self.backend.get(NODE_METRICS, name)
        except (ApiError, OSError) as e:
            log.warning("Failed to get metrics for node %s: %s", name, e)
            m = None
        return build_node_metrics(node, m)


def build_node_metrics(node: dict, metric: Optional[dict]) -> NodeMetrics:
    st = node.get("status", {})
    cap, alloc = st.get("capacity") or {}, st.get("allocatable") or {}
    cpu_cap = _q(cap, "cpu", True) or 0
    mem_cap = _q(cap, "memory", False) or 0
    disk_cap = _q(cap, "ephemeral-storage", False) or 0
    cpu_use = mem_use = 0
    if metric is not None:
        cpu_use = _q(metric.get("usage"), "cpu", True) or 0
        mem_use = _q(metric.get("usage"), "memory", False) or 0
    disk_use = 0
    a = _q(alloc, "ephemeral-storage", False)
    if a is not None:
        disk_use = max(0, disk_cap - a)
    healthy, conditions = True, None
    for c in st.get("conditions") or []:
        t, s, msg = c.get("type"), c.get("status"), c.get("message", "")
        if t == "Ready":
            if s != "True":
                healthy = False
                (conditions := conditions or []).append(f"NotReady: {msg}")
        elif s == "True" and t in ("MemoryPressure", "DiskPressure", "PIDPressure", "NetworkUnavailable"):
            healthy = False
            (conditions := conditions or []).append(f"{t}: {msg}")
    return NodeMetrics(
        node_name=node["metadata"]["name"], timestamp=utcnow(),
        cpu_capacity=cpu_cap, cpu_usage=cpu_use, cpu_usage_rate=cpu_use / cpu_cap * 100.0 if cpu_cap > 0 else 0.0,
        memory_capacity=mem_cap, memory_usage=mem_use,
        memory_usage_rate=mem_use / mem_cap * 100.0 if mem_cap > 0 else 0.0,
        disk_capacity=disk_cap, disk_usage=disk_use,
        disk_usage_rate=disk_use / disk_cap * 100.0 if disk_cap > 0 else 0.0,
        network_latency=0.0, network_bandwidth=0.0, gpu_count=0, gpu_models=[], gpu_usage=[], gpu_memory_total=[],
        gpu_memory_used=[], healthy=healthy, conditions=conditions,
        labels=dict(node["metadata"].get("labels") or {}), custom_metrics={})


class PodSource:
    def __init__(self, backend: ClusterBackend, namespaces: list[str]):
        self.backend = backend
        self.namespaces = namespaces

    def collect(self) -> dict:
        out: dict = {}
        for ns in self.namespaces:  # serial per namespace, like the reference
            try:
                out.update(self.collect_namespace(ns))
            except (ApiError, OSError) as e:
                log.warning("Failed to collect pod metrics for namespace %s: %s", ns, e)
        return out

    def collect_namespace(self, ns: str) -> dict:
        pods = self.backend.list(PODS, ns or None)
        try:
            pm = {m["metadata"]["name"]: m for m in self.backend.list(POD_METRICS, ns or None)}
        except (ApiError, OSError) as e:
            log.warning("Failed to get pod metrics from metrics server for namespace %s: %s", ns, e)
            pm = {}
        return {f'{p["metadata"].get("namespace", "")}/{p["metadata"]["name"]}': build_pod_metrics(p, pm.get(p["metadata"]["name"]))
                for p in pods}


def build_pod_metrics(pod: dict, metric: Optional[dict]) -> PodMetrics:
    spec, st, md = pod.get("spec", {}), pod.get("status", {}), pod.get("metadata", {})
    cpu_req = cpu_lim = mem_req = mem_lim = 0
    res_by_name = {}
    for c in spec.get("containers") or []:
        r = c.get("resources") or {}
        req, lim = r.get("requests") or {}, r.get("limits") or {}
        res_by_name[c.get("name")] = (req, lim)
        cpu_req += _q(req, "cpu", True) or 0
        cpu_lim += _q(lim, "cpu", True) or 0
        mem_req += _q(req, "memory", False) or 0
        mem_lim += _q(lim, "memory", False) or 0
    cpu_use = mem_use = 0
    containers = None
    if metric is not None:
        for c in metric.get("containers") or []:
            u = c.get("usage") or {}
            cu, mu = _q(u, "cpu", True) or 0, _q(u, "memory", False) or 0
            cpu_use += cu
            mem_use += mu
            req, lim = res_by_name.get(c.get("name"), ({}, {}))
            (containers := containers or []).append(ContainerMetrics(
                name=c.get("name", ""), cpu_usage=cu, memory_usage=mu, cpu_request=_q(req, "cpu", True) or 0,
                cpu_limit=_q(lim, "cpu", True) or 0, memory_request=_q(req, "memory", False) or 0,
                memory_limit=_q(lim, "memory", False) or 0))
    restarts = sum(int(s.get("restartCount") or 0) for s in st.get("containerStatuses") or [])
    ready = any(c.get("type") == "Ready" and c.get("status") == "True" for c in st.get("conditions") or [])
    return PodMetrics(
        pod_name=md.get("name", ""), namespace=md.get("namespace", ""), node_name=spec.get("nodeName", ""),
        timestamp=utcnow(), cpu_usage=cpu_use, memory_usage=mem_use, cpu_request=cpu_req, cpu_limit=cpu_lim,
        memory_request=mem_req, memory_limit=mem_lim,
        cpu_usage_rate=cpu_use / cpu_lim * 100.0 if cpu_lim > 0 else 0.0,
        memory_usage_rate=mem_use / mem_lim * 100.0 if mem_lim > 0 else 0.0,
        containers=containers, phase=st.get("phase", ""), ready=ready, restarts=restarts,
        start_time=parse_time(st.get("startTime")) or ZERO_TIME)


@dataclass
class PodPair:
    source_namespace: str
    source_pod: str
    source_ip: str
    target_namespace: str
    target_pod: str
    target_ip: str


class NetworkSource:
    def __init__(self, backend: ClusterBackend, tester, namespaces: list[str], max_pairs: int = 10,
                 test_timeout_s: float = 10.0, concurrency: int = 3, enable_auto_test: bool = True):
        self.backend, self.tester, self.namespaces = backend, tester, namespaces
        self.max_pairs = max_pairs if max_pairs > 0 else 10
        self.timeout = test_timeout_s
        self.concurrency = concurrency
        self.enable_auto_test = enable_auto_test

    def select_pairs(self) -> list[PodPair]:
        if not self.enable_auto_test:
            return []
        pods = []
        for ns in self.namespaces:
            try:
                for p in self.backend.list(PODS, ns or None, field_selector="status.phase=Running"):
                    if p.get("status", {}).get("podIP"):
                        pods.append(p)
            except (ApiError, OSError) as e:
                log.warning("Failed to list pods in namespace %s: %s", ns, e)
        if len(pods) < 2:
            return []

        def pair(a, b):
            return PodPair(a["metadata"]["namespace"], a["metadata"]["name"], a["status"]["podIP"],
                           b["metadata"]["namespace"], b["metadata"]["name"], b["status"]["podIP"])

        pairs = []
        for i in range(len(pods)):
            for j in range(i + 1, len(pods)):
                if len(pairs) >= self.max_pairs:
                    break
                if pods[i]["spec"].get("nodeName") != pods[j]["spec"].get("nodeName"):
                    pairs.append(pair(pods[i], pods[j]))
        if not pairs:
            for i in range(len(pods)):
                for j in range(i + 1, len(pods)):
                    if len(pairs) >= self.max_pairs:
                        break
                    pairs.append(pair(pods[i], pods[j]))
        return pairs

    def test_pair(self, p: PodPair) -> NetworkMetrics:
        m = NetworkMetrics(source_pod=f"{p.source_namespace}/{p.source_pod}",
                           target_pod=f"{p.target_namespace}/{p.target_pod}", timestamp=utcnow(), connected=False,
                           test_method="mixed")
        if self.tester is None:
            m.error = "K8s client not available"
            return m
        try:
            r = self.tester.test_pod_connectivity(m.source_pod, m.target_pod, timeout_s=self.timeout)
        except Exception as e:  # noqa: BLE001 - per-pair error isolation
            m.error = f"connectivity test failed: {e}"
            return m
        if r.success_rate > 0:
            m.connected = True
            m.rtt = r.average_rtt
            for x in r.rtt_results or []:
                if x.method == "ping" and x.success:
                    m.packet_loss = x.packet_loss
                    m.test_method = "ping"
                    break
            for x in r.rtt_results or []:
                if x.method == "http" and x.success:
                    m.rtt = x.rtt
                    m.test_method = "http"
                    break
        else:
            m.error = "all tests failed"
        return m

    def collect(self) -> list:
        pairs = self.select_pairs()
        if not pairs:
            return []
        with cf.ThreadPoolExecutor(max_workers=self.concurrency) as ex:  # semaphore of 3
            return [r for r in ex.map(self.test_pair, pairs) if r is not None]

    def test_pod_connectivity(self, source: str, target: str) -> NetworkMetrics:
        sns, sname = parse_pod_name_strict(source)
        tns, tname = parse_pod_name_strict(target)
        s = self.backend.get(PODS, sname, sns)
        t = self.backend.get(PODS, tname, tns)
        return self.test_pair(PodPair(sns, sname, s["status"].get("podIP", ""), tns, tname,
                                      t["status"].get("podIP", "")))


def parse_pod_name_strict(full: str) -> tuple[str, str]:
    """network_metrics.go:328-350: exactly two non-empty '/'-separated parts."""
    parts = [p for p in full.split("/") if p]
    if len(parts) != 2:
        raise ValueError("invalid pod name format, expected namespace/pod-name")
    return parts[0], parts[1]


class UAVSource:
    def __init__(self, backend: ClusterBackend, namespace: str = "default", label: str = "app=uav-agent",
                 timeout_s: float = 5.0):
        self.backend = backend
        self.namespace = namespace or "default"
        self.label = label or "app=uav-agent"
        self.timeout = timeout_s or 5.0

    def _agent_pods(self, node: Optional[str] = None) -> list:
        fs = "status.phase=Running" + (f",spec.nodeName={node}" if node else "")
        return self.backend.list(PODS, self.namespace, label_selector=self.label, field_selector=fs)

    def collect_single_pod(self, pod: dict) -> UAVState:
        ip = pod.get("status", {}).get("podIP")
        if not ip:
            raise RuntimeError(f"pod {pod['metadata']['name']} has no IP")
        code, body = self.backend.http_request("GET", f"http://{ip}:9090/api/v1/state", timeout_s=self.timeout)
        if code != 200:
            raise RuntimeError(f"unexpected status code: {code}")
        d = json.loads(body)
        if not isinstance(d, dict) or not d.get("data"):
            raise RuntimeError("no data in response")
        return UAVState.from_dict(d["data"])

    def collect(self) -> dict:
        pods = self._agent_pods()
        if not pods:
            log.warning("No running UAV agent pods found")
            return {}
        out = {}
        with cf.ThreadPoolExecutor(max_workers=min(64, len(pods))) as ex:  # one request per agent, concurrently
            futs = {ex.submit(self.collect_single_pod, p): p for p in pods}
            for f, p in futs.items():
                try:
                    out[p["spec"].get("nodeName", "")] = f.result()
                except Exception as e:  # noqa: BLE001 - a failing agent is skipped
                    log.warning("Failed to collect UAV metrics from node %s: %s", p["spec"].get("nodeName"), e)
        return out

    def collect_single(self, node: str) -> UAVState:
        pods = self._agent_pods(node)
        if not pods:
            raise RuntimeError(f"no UAV agent found on node {node}")
        return self.collect_single_pod(pods[0])

    def healthy_count(self) -> int:
        return sum(1 for s in self.collect().values() if s.health.system_status == "OK")

    def low_battery(self, threshold: float) -> list[str]:
        return [n for n, s in self.collect().items() if s.battery.remaining_percent < threshold]

    def send_command(self, node: str, command: str, payload: Optional[dict] = None) -> dict:
        """Unlike uav_metrics.go:239-287 (which drops the payload), the JSON body is sent."""
        pods = self._agent_pods(node)
        if not pods:
            raise RuntimeError(f"no UAV agent found on node {node}")
        body = json.dumps(payload).encode() if payload is not None else None
        code, data = self.backend.http_request("POST", f"http://{pods[0]['status']['podIP']}:9090/api/v1/command/{command}",
                                               body=body, timeout_s=self.timeout)
        if code != 200:
            raise RuntimeError(f"command failed with status: {code}")
        return json.loads(data)
