"""``k8s.Client`` equivalent (``internal/k8s/client.go:25-480``, K1) and the object converters
(``internal/k8s/converter.go:13-119``, K2), over any :class:`ClusterBackend`.
"""
from __future__ import annotations

import logging
from typing import Optional

from ...utils.gojson import ZERO_TIME, format_time_rfc3339, parse_time, utcnow
from ..config import K8sConfig, parse_namespaces
from ..types import ContainerInfo, CustomResourceInfo, EventInfo, PodInfo, ServiceInfo, ServicePort, UAVReport
from .backend import EVENTS, NODES, PODS, SERVICES, UAV_METRICS, ApiError, ClusterBackend

log = logging.getLogger("k8s")


# --------------------------------------------------------------------------- converters (K2)

def _container_state(status: Optional[dict]) -> str:
    if status is None:
        return "Unknown"
    st = status.get("state") or {}
    if st.get("running") is not None:
        return "Running"
    if st.get("waiting") is not None:
        return "Waiting"
    if st.get("terminated") is not None:
        return "Terminated"
    return "Unknown"


def convert_pod(pod: dict) -> PodInfo:
    """convertPodToModel (converter.go:13-47).  Env keeps literal values only (valueFrom skipped)."""
    md, spec, st = pod.get("metadata", {}), pod.get("spec", {}), pod.get("status", {})
    statuses = {s.get("name"): s for s in st.get("containerStatuses") or []}
    containers = None
    for c in spec.get("containers") or []:
        cs = statuses.get(c.get("name"))
        env = {e["name"]: e["value"] for e in c.get("env") or [] if e.get("value")}
        (containers := containers or []).append(ContainerInfo(
            name=c.get("name", ""), image=c.get("image", ""), state=_container_state(cs),
            ready=bool(cs and cs.get("ready")), env=env))
    return PodInfo(name=md.get("name", ""), namespace=md.get("namespace", ""), status=st.get("phase", ""),
                   node_name=spec.get("nodeName", ""), ip=st.get("podIP", ""), labels=md.get("labels") or None,
                   start_time=parse_time(md.get("creationTimestamp")) or ZERO_TIME, containers=containers)


def convert_service(svc: dict) -> ServiceInfo:
    md, spec = svc.get("metadata", {}), svc.get("spec", {})
    ports = None
    for p in spec.get("ports") or []:
        (ports := ports or []).append(ServicePort(name=p.get("name", ""), port=int(p.get("port", 0)),
                                                  protocol=p.get("protocol", "")))
    return ServiceInfo(name=md.get("name", ""), namespace=md.get("namespace", ""), type=spec.get("type", ""),
                       cluster_ip=spec.get("clusterIP", ""), ports=ports, selector=spec.get("selector") or None)


def convert_event(ev: dict) -> EventInfo:
    return EventInfo(type=ev.get("type", ""), reason=ev.get("reason", ""), message=ev.get("message", ""),
                     source=(ev.get("source") or {}).get("component", ""),
                     timestamp=parse_time(ev.get("lastTimestamp")) or ZERO_TIME, count=int(ev.get("count") or 0))


def last_update_time(obj: dict):
    """getLastUpdateTime (client.go:463-471): managedFields[0].time, else creation."""
    md = obj.get("metadata", {})
    mf = md.get("managedFields") or []
    if mf and mf[0].get("time"):
        return parse_time(mf[0]["time"]) or ZERO_TIME
    return parse_time(md.get("creationTimestamp")) or ZERO_TIME


def convert_custom_resource(obj: dict, group: str, kind: str) -> CustomResourceInfo:
    """convertUnstructuredToModel (client.go:290-313); a missing/non-map spec or status becomes {}."""
    md = obj.get("metadata", {})
    spec = obj.get("spec") if isinstance(obj.get("spec"), dict) else {}
    status = obj.get("status") if isinstance(obj.get("status"), dict) else {}
    return CustomResourceInfo(kind=kind, name=md.get("name", ""), namespace=md.get("namespace", ""), group=group,
                              version=obj.get("apiVersion", ""), spec=spec, status=status,
                              generation=int(md.get("generation") or 0),
                              creation_time=parse_time(md.get("creationTimestamp")) or ZERO_TIME,
                              update_time=last_update_time(obj))


def sanitize_resource_name(name: str) -> str:
    """client.go:452-461: lowercase, ``_`` and ``.`` -> ``-``, trimmed, empty -> "unknown"."""
    n = name.lower().replace("_", "-").replace(".", "-").strip()
    return n or "unknown"


# --------------------------------------------------------------------------- client (K1)

class K8sClient:
    def __init__(self, backend: ClusterBackend, cfg: Optional[K8sConfig] = None):
        self.backend = backend
        self.cfg = cfg or K8sConfig()
        self.namespaces = parse_namespaces(self.cfg.watch_namespaces)

    # TestConnection (client.go:103-112)
    def test_connection(self) -> str:
        v = self.backend.server_version()
        return v.get("gitVersion", "")

    def server_version(self) -> str:
        return self.backend.server_version().get("gitVersion", "")

    def get_cluster_info(self) -> dict:
        """GetClusterInfo (client.go:115-150): version, node count, pods in watched namespaces."""
        version = self.server_version()
        nodes = self.backend.list(NODES)
        pods = 0
        for ns in self.namespaces:
            try:
                pods += len(self.backend.list(PODS, ns))
            except (ApiError, OSError) as e:
                log.warning("Failed to list pods in namespace %s: %s", ns, e)
        return {"version": version, "nodes": len(nodes), "pods": pods, "namespaces": list(self.namespaces)}

    def get_pods(self, namespace: str) -> Optional[list]:
        return [convert_pod(p) for p in self.backend.list(PODS, namespace)] or None

    def get_pod(self, namespace: str, name: str) -> PodInfo:
        return convert_pod(self.backend.get(PODS, name, namespace))

    def get_services(self, namespace: str) -> Optional[list]:
        return [convert_service(s) for s in self.backend.list(SERVICES, namespace)] or None

    def get_events(self, namespace: str, limit: int = 0) -> Optional[list]:
        return [convert_event(e) for e in self.backend.list(EVENTS, namespace, limit=limit)] or None

    def get_pod_logs(self, namespace: str, pod: str, lines: int = 100) -> str:
        return self.backend.pod_logs(namespace, pod, lines)

    # ---------------------------------------------------------------- UAVMetric CRD (K1c, K1d)
    def list_uav_metrics_crd(self, namespace: str = "") -> list:
        objs = self.backend.list(UAV_METRICS, namespace or None)
        return [convert_custom_resource(o, "monitoring.io", "UAVMetric") for o in objs]

    def upsert_uav_metric(self, report: UAVReport, namespace: str = "") -> str:
        """UpsertUAVMetric (client.go:316-450).  Returns "created" | "updated"."""
        if report is None:
            raise ValueError("uav report is nil")
        if not report.node_name:
            raise ValueError("uav report missing node name")
        namespace = namespace or self.cfg.namespace or "default"
        name = f"uavmetric-{sanitize_resource_name(report.node_name)}"
        ts = report.timestamp if report.timestamp and report.timestamp != ZERO_TIME else utcnow()
        spec: dict = {"node_name": report.node_name, "uav_id": report.uav_id}
        s = report.state
        if s is not None:
            spec["gps"] = {"latitude": s.gps.latitude, "longitude": s.gps.longitude, "altitude": s.gps.altitude,
                           "relative_altitude": s.gps.relative_altitude, "satellite_count": s.gps.satellite_count,
                           "fix_type": s.gps.fix_type}
            spec["battery"] = {"voltage": s.battery.voltage, "remaining_percent": s.battery.remaining_percent,
                               "remaining_capacity": s.battery.remaining_capacity,
                               "temperature": s.battery.temperature}
            spec["flight"] = {"mode": s.flight.mode, "armed": s.flight.armed, "ground_speed": s.flight.ground_speed,
                              "vertical_speed": s.flight.vertical_speed}
            spec["health"] = {"system_status": s.health.system_status, "error_count": s.health.error_count,
                              "warning_count": s.health.warning_count}
        status = {"last_update": format_time_rfc3339(ts), "collection_status": report.status or "active"}
        labels = {"app": "uav-agent", "monitoring.io/component": "uav-metrics",
                  "monitoring.io/node": sanitize_resource_name(report.node_name)}
        if report.uav_id:
            labels["monitoring.io/uav-id"] = sanitize_resource_name(report.uav_id)
        if report.node_ip:
            labels["monitoring.io/node-ip"] = report.node_ip
        try:
            existing = self.backend.get(UAV_METRICS, name, namespace)
        except ApiError as e:
            if not e.not_found:
                raise RuntimeError(f"failed to get UAVMetric {name}: {e}") from e
            obj = {"apiVersion": "monitoring.io/v1", "kind": "UAVMetric",
                   "metadata": {"name": name, "namespace": namespace, "labels": labels},
                   "spec": spec, "status": status}
            try:
                self.backend.create(UAV_METRICS, obj, namespace)
            except ApiError as ce:
                raise RuntimeError(f"failed to create UAVMetric {name}: {ce}") from ce
            return "created"
        existing["spec"] = spec
        existing["status"] = status  # no status subresource on this CRD: plain update carries it
        md = existing.setdefault("metadata", {})
        if isinstance(md.get("labels"), dict):
            md["labels"].update(labels)
        else:
            md["labels"] = labels
        try:
            self.backend.update(UAV_METRICS, existing, namespace)
        except ApiError as ue:
            raise RuntimeError(f"failed to update UAVMetric {name}: {ue}") from ue
        return "updated"
