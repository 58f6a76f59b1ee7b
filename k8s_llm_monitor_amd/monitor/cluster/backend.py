"""Cluster access abstraction (replaces the reference's client-go clientsets).

Objects are raw Kubernetes JSON (``dict``), exactly what the API server returns, so the same
converters run against a live cluster (:class:`KubeRESTBackend`) and the deterministic in-memory
:class:`FakeCluster`.  Resources are addressed by :class:`GVR` like the dynamic client.
"""
from __future__ import annotations

import re
from abc import ABC, abstractmethod
from typing import Iterator, NamedTuple, Optional


class GVR(NamedTuple):
    group: str
    version: str
    resource: str
    namespaced: bool = True

    @property
    def api_version(self) -> str:
        return f"{self.group}/{self.version}" if self.group else self.version


PODS = GVR("", "v1", "pods")
SERVICES = GVR("", "v1", "services")
EVENTS = GVR("", "v1", "events")
NODES = GVR("", "v1", "nodes", False)
NAMESPACES = GVR("", "v1", "namespaces", False)
NETWORK_POLICIES = GVR("networking.k8s.io", "v1", "networkpolicies")
NODE_METRICS = GVR("metrics.k8s.io", "v1beta1", "nodes", False)
POD_METRICS = GVR("metrics.k8s.io", "v1beta1", "pods")
CRDS = GVR("apiextensions.k8s.io", "v1", "customresourcedefinitions", False)
UAV_METRICS = GVR("monitoring.io", "v1", "uavmetrics")
SCHEDULING_REQUESTS = GVR("scheduler.io", "v1", "schedulingrequests")

KINDS = {PODS: "Pod", SERVICES: "Service", EVENTS: "Event", NODES: "Node", NAMESPACES: "Namespace",
         NETWORK_POLICIES: "NetworkPolicy", NODE_METRICS: "NodeMetrics", POD_METRICS: "PodMetrics",
         CRDS: "CustomResourceDefinition", UAV_METRICS: "UAVMetric", SCHEDULING_REQUESTS: "SchedulingRequest"}


class ApiError(Exception):
    """A Kubernetes API ``Status`` failure (``reason`` e.g. NotFound, AlreadyExists, Conflict)."""

    def __init__(self, code: int, reason: str, message: str):
        super().__init__(message)
        self.code, self.reason, self.message = code, reason, message

    @property
    def not_found(self) -> bool:
        return self.code == 404 or self.reason == "NotFound"


class ExecError(Exception):
    pass


class ClusterBackend(ABC):
    """What the monitor needs from a cluster.  Every method may raise :class:`ApiError` or
    ``OSError`` (unreachable API server)."""

    @abstractmethod
    def server_version(self) -> dict: ...

    @abstractmethod
    def list(self, gvr: GVR, namespace: Optional[str] = None, label_selector: str = "",
             field_selector: str = "", limit: int = 0) -> list[dict]: ...

    @abstractmethod
    def get(self, gvr: GVR, name: str, namespace: Optional[str] = None) -> dict: ...

    @abstractmethod
    def create(self, gvr: GVR, obj: dict, namespace: Optional[str] = None) -> dict: ...

    @abstractmethod
    def update(self, gvr: GVR, obj: dict, namespace: Optional[str] = None) -> dict: ...

    @abstractmethod
    def update_status(self, gvr: GVR, obj: dict, namespace: Optional[str] = None) -> dict: ...

    @abstractmethod
    def delete(self, gvr: GVR, name: str, namespace: Optional[str] = None) -> None: ...

    @abstractmethod
    def watch(self, gvr: GVR, namespace: Optional[str] = None, resource_version: str = "",
              timeout_s: float = 300.0, stop=None) -> Iterator[tuple[str, dict]]:
        """Yields (event type ADDED|MODIFIED|DELETED|BOOKMARK|ERROR, object) until the stream ends."""

    @abstractmethod
    def exec(self, namespace: str, pod: str, container: str, command: list[str],
             timeout_s: float = 30.0) -> tuple[str, str]:
        """Run ``command`` in a container (pods/exec); returns (stdout, stderr)."""

    @abstractmethod
    def pod_logs(self, namespace: str, pod: str, tail_lines: int = 100) -> str: ...

    @abstractmethod
    def http_request(self, method: str, url: str, body: Optional[bytes] = None,
                     timeout_s: float = 5.0) -> tuple[int, bytes]:
        """An HTTP request to an in-cluster endpoint (UAV agents on pod IPs)."""


# --------------------------------------------------------------------------- selectors

_SET_RE = re.compile(r"^\s*([A-Za-z0-9_./-]+)\s+(in|notin)\s+\(([^)]*)\)\s*$")


def _split_selector(sel: str) -> list[str]:
    parts, depth, cur = [], 0, ""
    for ch in sel:
        if ch == "(":
            depth += 1
        elif ch == ")":
            depth -= 1
        if ch == "," and depth == 0:
            parts.append(cur)
            cur = ""
        else:
            cur += ch
    if cur.strip():
        parts.append(cur)
    return [p.strip() for p in parts if p.strip()]


def match_labels(selector: str, labels: Optional[dict]) -> bool:
    """Kubernetes label-selector semantics (=, ==, !=, in, notin, exists, !exists)."""
    labels = labels or {}
    for req in _split_selector(selector or ""):
        m = _SET_RE.match(req)
        if m:
            key, op, vals = m.group(1), m.group(2), {v.strip() for v in m.group(3).split(",") if v.strip()}
            if op == "in" and labels.get(key) not in vals:
                return False
            if op == "notin" and key in labels and labels[key] in vals:
                return False
            continue
        if "!=" in req:
            k, v = (x.strip() for x in req.split("!=", 1))
            if labels.get(k) == v:
                return False
        elif "==" in req or "=" in req:
            k, v = (x.strip() for x in req.replace("==", "=").split("=", 1))
            if labels.get(k) != v:
                return False
        elif req.startswith("!"):
            if req[1:].strip() in labels:
                return False
        elif req not in labels:
            return False
    return True


def _field(obj: dict, path: str):
    cur = obj
    for p in path.split("."):
        if not isinstance(cur, dict):
            return None
        cur = cur.get(p)
    return cur


def match_fields(selector: str, obj: dict) -> bool:
    """Field selectors as the API server supports them (``a.b=v``, ``a.b!=v``, comma-AND)."""
    for req in _split_selector(selector or ""):
        neg = "!=" in req
        k, v = (x.strip() for x in req.replace("==", "=").split("!=" if neg else "=", 1))
        val = _field(obj, k)
        val = "" if val is None else str(val)
        if (val == v) == neg:
            return False
    return True


# --------------------------------------------------------------------------- quantities

_SUFFIX = {"n": 1e-9, "u": 1e-6, "m": 1e-3, "": 1, "k": 1e3, "M": 1e6, "G": 1e9, "T": 1e12, "P": 1e15, "E": 1e18,
           "Ki": 2 ** 10, "Mi": 2 ** 20, "Gi": 2 ** 30, "Ti": 2 ** 40, "Pi": 2 ** 50, "Ei": 2 ** 60}
_Q_RE = re.compile(r"^([+-]?[0-9.]+)([eE][+-]?[0-9]+)?(Ki|Mi|Gi|Ti|Pi|Ei|n|u|m|k|M|G|T|P|E)?$")


def parse_quantity(q) -> float:
    """resource.Quantity -> float base units (cores, bytes)."""
    if q is None:
        return 0.0
    if isinstance(q, (int, float)):
        return float(q)
    m = _Q_RE.match(str(q).strip())
    if not m:
        raise ValueError(f"invalid quantity {q!r}")
    num = float(m.group(1) + (m.group(2) or ""))
    return num * _SUFFIX[m.group(3) or ""]


def milli_value(q) -> int:
    """``Quantity.MilliValue()`` (rounds up, like the apimachinery implementation)."""
    import math

    return int(math.ceil(round(parse_quantity(q) * 1000.0, 6)))


def value(q) -> int:
    """``Quantity.Value()`` (rounds up)."""
    import math

    return int(math.ceil(round(parse_quantity(q), 6)))
