"""API data models, field-for-field with the reference's JSON contracts.

* ``pkg/models/models.go:10-192``   -> PodInfo ... UAVReport (D1)
* ``pkg/models/scheduler.go:6-38``  -> SchedulingWorkload ... SchedulingCandidate (D2)
* ``pkg/metrics/types.go:8-199``    -> NodeMetrics ... MetricsSnapshot + helper methods (D3)
* ``pkg/uav/mavlink_simulator.go:11-106`` -> UAVState and its sub-structs

Field order is declaration order (Go struct order); JSON names / omitempty come from the Go
struct tags.  Slices/maps that Go leaves nil default to None here (encoded ``null``).
"""
from __future__ import annotations

import copy
import datetime as _dt
from dataclasses import dataclass, fields
from typing import Any, Optional

from ..utils.gojson import jfield, parse_time


def _from_dict(cls, d: Optional[dict]):
    """Decode a JSON object into a dataclass the way Go's json.Unmarshal would (unknown keys
    ignored, missing keys left at their zero value, nested dataclasses / times decoded)."""
    if d is None:
        return None
    if not isinstance(d, dict):
        raise ValueError(f"expected JSON object for {cls.__name__}")
    kw = {}
    hints = getattr(cls, "_nested", {})
    for f in fields(cls):
        name = f.metadata.get("json") or f.name
        if name not in d:
            continue
        v = d[name]
        sub = hints.get(f.name)
        if f.metadata.get("time"):
            v = parse_time(v) if isinstance(v, str) else None
        elif sub is not None:
            if isinstance(sub, list):
                v = [_from_dict(sub[0], x) for x in v] if isinstance(v, list) else None
            else:
                v = _from_dict(sub, v)
        kw[f.name] = v
    return cls(**kw)


# --------------------------------------------------------------------------- pkg/models


@dataclass
class ContainerInfo:
    name: str = jfield("name", default="")
    image: str = jfield("image", default="")
    state: str = jfield("state", default="")
    ready: bool = jfield("ready", default=False)
    env: Optional[dict] = jfield("env")


@dataclass
class PodInfo:
    name: str = jfield("name", default="")
    namespace: str = jfield("namespace", default="")
    status: str = jfield("status", default="")
    node_name: str = jfield("node_name", default="")
    ip: str = jfield("ip", default="")
    labels: Optional[dict] = jfield("labels")
    start_time: Optional[_dt.datetime] = jfield("start_time", time=True)
    containers: Optional[list] = jfield("containers")


@dataclass
class ServicePort:
    name: str = jfield("name", default="")
    port: int = jfield("port", default=0)
    protocol: str = jfield("protocol", default="")


@dataclass
class ServiceInfo:
    name: str = jfield("name", default="")
    namespace: str = jfield("namespace", default="")
    type: str = jfield("type", default="")
    cluster_ip: str = jfield("cluster_ip", default="")
    ports: Optional[list] = jfield("ports")
    selector: Optional[dict] = jfield("selector")


@dataclass
class EventInfo:
    type: str = jfield("type", default="")
    reason: str = jfield("reason", default="")
    message: str = jfield("message", default="")
    source: str = jfield("source", default="")
    timestamp: Optional[_dt.datetime] = jfield("timestamp", time=True)
    count: int = jfield("count", default=0)


@dataclass
class PortRule:
    protocol: str = jfield("protocol", default="")
    port: int = jfield("port", default=0)


@dataclass
class PeerRule:
    pod_selector: Optional[dict] = jfield("pod_selector")
    namespace_selector: Optional[dict] = jfield("namespace_selector")


@dataclass
class NetworkPolicyRule:
    ports: Optional[list] = jfield("ports")
    from_: Optional[list] = jfield("from")
    to: Optional[list] = jfield("to")


@dataclass
class NetworkPolicyInfo:
    name: str = jfield("name", default="")
    namespace: str = jfield("namespace", default="")
    pod_selector: Optional[dict] = jfield("pod_selector")
    ingress: Optional[list] = jfield("ingress")
    egress: Optional[list] = jfield("egress")


@dataclass
class AnalysisRequest:
    """``type`` is "pod_communication" | "anomaly_detection" | "root_cause" (models.go:87)."""
    type: str = jfield("type", default="")
    parameters: Optional[dict] = jfield("parameters")
    context: Optional[dict] = jfield("context")


@dataclass
class AnalysisResponse:
    request_id: str = jfield("request_id", default="")
    status: str = jfield("status", default="")  # success | error | processing
    result: Optional[dict] = jfield("result")
    error: str = jfield("error", omitempty=True, default="")
    timestamp: Optional[_dt.datetime] = jfield("timestamp", time=True)


@dataclass
class CommunicationAnalysis:
    pod_a: str = jfield("pod_a", default="")
    pod_b: str = jfield("pod_b", default="")
    status: str = jfield("status", default="unknown")
    issues: Optional[list] = jfield("issues")
    solutions: Optional[list] = jfield("solutions")
    confidence: float = jfield("confidence", default=0.0)


@dataclass
class SystemHealth:
    overall_health: str = jfield("overall_health", default="")
    components: Optional[dict] = jfield("components")
    issues: Optional[list] = jfield("issues")
    suggestions: Optional[list] = jfield("suggestions")
    last_update: Optional[_dt.datetime] = jfield("last_update", time=True)


@dataclass
class CRDInfo:
    name: str = jfield("name", default="")
    group: str = jfield("group", default="")
    kind: str = jfield("kind", default="")
    scope: str = jfield("scope", default="")
    versions: Optional[list] = jfield("versions")
    plural: str = jfield("plural", default="")
    singular: str = jfield("singular", default="")
    established: bool = jfield("established", default=False)
    stored: bool = jfield("stored", default=False)
    creation_time: Optional[_dt.datetime] = jfield("creation_time", time=True)


@dataclass
class CustomResourceInfo:
    kind: str = jfield("kind", default="")
    name: str = jfield("name", default="")
    namespace: str = jfield("namespace", default="")
    group: str = jfield("group", default="")
    version: str = jfield("version", default="")
    spec: Optional[dict] = jfield("spec")
    status: Optional[dict] = jfield("status")
    generation: int = jfield("generation", default=0)
    creation_time: Optional[_dt.datetime] = jfield("creation_time", time=True)
    update_time: Optional[_dt.datetime] = jfield("update_time", time=True)


@dataclass
class CRDEvent:
    type: str = jfield("type", default="")  # ADDED / MODIFIED / DELETED
    kind: str = jfield("kind", default="")
    group: str = jfield("group", default="")
    version: str = jfield("version", default="")
    name: str = jfield("name", default="")
    namespace: str = jfield("namespace", default="")
    object: Optional[dict] = jfield("object")
    timestamp: Optional[_dt.datetime] = jfield("timestamp", time=True)


@dataclass
class RTTResult:
    success: bool = jfield("success", default=False)
    rtt: float = jfield("rtt_ms", default=0.0)
    packet_loss: float = jfield("packet_loss", default=0.0)
    error_message: str = jfield("error_message", default="")
    timestamp: Optional[_dt.datetime] = jfield("timestamp", time=True)
    method: str = jfield("method", default="")


@dataclass
class NetworkTestResult:
    pod_a: str = jfield("pod_a", default="")
    pod_b: str = jfield("pod_b", default="")
    rtt_results: Optional[list] = jfield("rtt_results")
    average_rtt: float = jfield("average_rtt_ms", default=0.0)
    success_rate: float = jfield("success_rate", default=0.0)
    test_count: int = jfield("test_count", default=0)
    latency: str = jfield("latency_assessment", default="")


# --------------------------------------------------------------------------- pkg/uav


@dataclass
class GPSData:
    latitude: float = jfield("latitude", default=0.0)
    longitude: float = jfield("longitude", default=0.0)
    altitude: float = jfield("altitude", default=0.0)
    relative_altitude: float = jfield("relative_altitude", default=0.0)
    hdop: float = jfield("hdop", default=0.0)
    satellite_count: int = jfield("satellite_count", default=0)
    fix_type: int = jfield("fix_type", default=0)
    ground_speed: float = jfield("ground_speed", default=0.0)
    course_over_ground: float = jfield("course_over_ground", default=0.0)
    timestamp: Optional[_dt.datetime] = jfield("timestamp", time=True)


@dataclass
class AttitudeData:
    roll: float = jfield("roll", default=0.0)
    pitch: float = jfield("pitch", default=0.0)
    yaw: float = jfield("yaw", default=0.0)
    roll_rate: float = jfield("roll_rate", default=0.0)
    pitch_rate: float = jfield("pitch_rate", default=0.0)
    yaw_rate: float = jfield("yaw_rate", default=0.0)
    timestamp: Optional[_dt.datetime] = jfield("timestamp", time=True)


@dataclass
class FlightData:
    mode: str = jfield("mode", default="")
    armed: bool = jfield("armed", default=False)
    airspeed: float = jfield("airspeed", default=0.0)
    ground_speed: float = jfield("ground_speed", default=0.0)
    vertical_speed: float = jfield("vertical_speed", default=0.0)
    throttle_percent: float = jfield("throttle_percent", default=0.0)
    timestamp: Optional[_dt.datetime] = jfield("timestamp", time=True)


@dataclass
class BatteryData:
    voltage: float = jfield("voltage", default=0.0)
    current: float = jfield("current", default=0.0)
    remaining_percent: float = jfield("remaining_percent", default=0.0)
    remaining_capacity: float = jfield("remaining_capacity", default=0.0)
    total_capacity: float = jfield("total_capacity", default=0.0)
    temperature: float = jfield("temperature", default=0.0)
    cell_count: int = jfield("cell_count", default=0)
    time_remaining: int = jfield("time_remaining", default=0)
    timestamp: Optional[_dt.datetime] = jfield("timestamp", time=True)


@dataclass
class MissionData:
    current_waypoint: int = jfield("current_waypoint", default=0)
    total_waypoints: int = jfield("total_waypoints", default=0)
    mission_state: str = jfield("mission_state", default="")
    distance_to_wp: float = jfield("distance_to_wp", default=0.0)
    eta_to_wp: int = jfield("eta_to_wp", default=0)
    timestamp: Optional[_dt.datetime] = jfield("timestamp", time=True)


@dataclass
class HealthData:
    system_status: str = jfield("system_status", default="")
    sensors_health: Optional[dict] = jfield("sensors_health")
    error_count: int = jfield("error_count", default=0)
    warning_count: int = jfield("warning_count", default=0)
    messages: Optional[list] = jfield("messages")
    last_heartbeat: Optional[_dt.datetime] = jfield("last_heartbeat", time=True)
    timestamp: Optional[_dt.datetime] = jfield("timestamp", time=True)


@dataclass
class UAVState:
    uav_id: str = jfield("uav_id", default="")
    node_name: str = jfield("node_name", default="")
    system_time: Optional[_dt.datetime] = jfield("system_time", time=True)
    gps: GPSData = jfield("gps", default_factory=GPSData)
    attitude: AttitudeData = jfield("attitude", default_factory=AttitudeData)
    flight: FlightData = jfield("flight", default_factory=FlightData)
    battery: BatteryData = jfield("battery", default_factory=BatteryData)
    mission: MissionData = jfield("mission", default_factory=MissionData)
    health: HealthData = jfield("health", default_factory=HealthData)

    _nested = {"gps": GPSData, "attitude": AttitudeData, "flight": FlightData, "battery": BatteryData,
               "mission": MissionData, "health": HealthData}

    def copy(self) -> "UAVState":
        """Deep copy (the reference's GetState copies the struct but shares the health map and
        message slice - SURVEY.md §5 race list; we do not)."""
        return copy.deepcopy(self)

    @classmethod
    def from_dict(cls, d: dict) -> "UAVState":
        return _from_dict(cls, d)


@dataclass
class UAVReport:
    node_name: str = jfield("node_name", default="")
    node_ip: str = jfield("node_ip", omitempty=True, default="")
    uav_id: str = jfield("uav_id", default="")
    source: str = jfield("source", default="")
    status: str = jfield("status", default="")
    timestamp: Optional[_dt.datetime] = jfield("timestamp", time=True)
    heartbeat_interval_seconds: int = jfield("heartbeat_interval_seconds", omitempty=True, default=0)
    state: Optional[UAVState] = jfield("state", omitempty=True)
    metadata: Optional[dict] = jfield("metadata", omitempty=True)

    _nested = {"state": UAVState}

    @classmethod
    def from_dict(cls, d: dict) -> "UAVReport":
        return _from_dict(cls, d)


# --------------------------------------------------------------------------- pkg/models/scheduler.go


@dataclass
class SchedulingWorkload:
    name: str = jfield("name", default="")
    namespace: str = jfield("namespace", default="")
    type: str = jfield("type", omitempty=True, default="")


@dataclass
class SchedulingRequestSpec:
    workload: SchedulingWorkload = jfield("workload", default_factory=SchedulingWorkload)
    min_battery_percent: float = jfield("minBatteryPercent", omitempty=True, default=0.0)
    preferred_nodes: Optional[list] = jfield("preferredNodes", omitempty=True)
    annotations: Optional[dict] = jfield("annotations", omitempty=True)
    created_at: Optional[_dt.datetime] = jfield("createdAt", omitempty=True)


@dataclass
class SchedulingRequestStatus:
    phase: str = jfield("phase", omitempty=True, default="")
    assigned_node: str = jfield("assignedNode", omitempty=True, default="")
    assigned_uav: str = jfield("assignedUAV", omitempty=True, default="")
    score: float = jfield("score", omitempty=True, default=0.0)
    message: str = jfield("message", omitempty=True, default="")
    last_updated: Optional[_dt.datetime] = jfield("lastUpdated", omitempty=True)


@dataclass
class SchedulingCandidate:
    node_name: str = ""
    uav_id: str = ""
    battery: float = 0.0
    last_heartbeat: Optional[_dt.datetime] = None
    score: float = 0.0


# --------------------------------------------------------------------------- pkg/metrics


@dataclass
class NodeMetrics:
    node_name: str = jfield("node_name", default="")
    timestamp: Optional[_dt.datetime] = jfield("timestamp", time=True)
    cpu_capacity: int = jfield("cpu_capacity", default=0)
    cpu_usage: int = jfield("cpu_usage", default=0)
    cpu_usage_rate: float = jfield("cpu_usage_rate", default=0.0)
    memory_capacity: int = jfield("memory_capacity", default=0)
    memory_usage: int = jfield("memory_usage", default=0)
    memory_usage_rate: float = jfield("memory_usage_rate", default=0.0)
    disk_capacity: int = jfield("disk_capacity", default=0)
    disk_usage: int = jfield("disk_usage", default=0)
    disk_usage_rate: float = jfield("disk_usage_rate", default=0.0)
    network_latency: float = jfield("network_latency", default=0.0)
    network_bandwidth: float = jfield("network_bandwidth", default=0.0)
    gpu_count: int = jfield("gpu_count", default=0)
    gpu_models: Optional[list] = jfield("gpu_models")
    gpu_usage: Optional[list] = jfield("gpu_usage")
    gpu_memory_total: Optional[list] = jfield("gpu_memory_total")
    gpu_memory_used: Optional[list] = jfield("gpu_memory_used")
    healthy: bool = jfield("healthy", default=False)
    conditions: Optional[list] = jfield("conditions")
    labels: Optional[dict] = jfield("labels")
    custom_metrics: Optional[dict] = jfield("custom_metrics", omitempty=True)

    def get_available_resources(self) -> tuple[float, float, float]:
        """(cpu cores, memory GiB, disk GiB) free (types.go:151-157)."""
        gib = 1024.0 ** 3
        return ((self.cpu_capacity - self.cpu_usage) / 1000.0, (self.memory_capacity - self.memory_usage) / gib,
                (self.disk_capacity - self.disk_usage) / gib)

    def is_under_pressure(self) -> bool:
        """CPU or memory > 80 %, or disk > 90 % (types.go:160-163)."""
        return self.cpu_usage_rate > 80.0 or self.memory_usage_rate > 80.0 or self.disk_usage_rate > 90.0


@dataclass
class ContainerMetrics:
    name: str = jfield("name", default="")
    cpu_usage: int = jfield("cpu_usage", default=0)
    memory_usage: int = jfield("memory_usage", default=0)
    cpu_request: int = jfield("cpu_request", default=0)
    cpu_limit: int = jfield("cpu_limit", default=0)
    memory_request: int = jfield("memory_request", default=0)
    memory_limit: int = jfield("memory_limit", default=0)


@dataclass
class PodMetrics:
    pod_name: str = jfield("pod_name", default="")
    namespace: str = jfield("namespace", default="")
    node_name: str = jfield("node_name", default="")
    timestamp: Optional[_dt.datetime] = jfield("timestamp", time=True)
    cpu_usage: int = jfield("cpu_usage", default=0)
    memory_usage: int = jfield("memory_usage", default=0)
    cpu_request: int = jfield("cpu_request", default=0)
    cpu_limit: int = jfield("cpu_limit", default=0)
    memory_request: int = jfield("memory_request", default=0)
    memory_limit: int = jfield("memory_limit", default=0)
    cpu_usage_rate: float = jfield("cpu_usage_rate", default=0.0)
    memory_usage_rate: float = jfield("memory_usage_rate", default=0.0)
    containers: Optional[list] = jfield("containers")
    phase: str = jfield("phase", default="")
    ready: bool = jfield("ready", default=False)
    restarts: int = jfield("restarts", default=0)
    start_time: Optional[_dt.datetime] = jfield("start_time", time=True)

    def get_resource_utilization(self) -> tuple[float, float]:
        """Usage relative to the *request* (types.go:166-174)."""
        cpu = self.cpu_usage / self.cpu_request * 100.0 if self.cpu_request > 0 else 0.0
        mem = self.memory_usage / self.memory_request * 100.0 if self.memory_request > 0 else 0.0
        return cpu, mem

    def is_over_limit(self) -> bool:
        """Usage >= 90 % of a limit (types.go:177-185); Go truncates limit*0.9 to int64."""
        if self.cpu_limit > 0 and self.cpu_usage >= int(self.cpu_limit * 0.9):
            return True
        if self.memory_limit > 0 and self.memory_usage >= int(self.memory_limit * 0.9):
            return True
        return False


@dataclass
class NetworkMetrics:
    source_pod: str = jfield("source_pod", default="")
    target_pod: str = jfield("target_pod", default="")
    timestamp: Optional[_dt.datetime] = jfield("timestamp", time=True)
    connected: bool = jfield("connected", default=False)
    error: str = jfield("error", omitempty=True, default="")
    rtt: float = jfield("rtt_ms", default=0.0)
    packet_loss: float = jfield("packet_loss", default=0.0)
    bandwidth: float = jfield("bandwidth_mbps", omitempty=True, default=0.0)
    test_method: str = jfield("test_method", default="")

    def get_quality(self) -> str:
        """<10 ms excellent, <50 good, <100 fair, else poor (types.go:188-199; differs from the RTT
        tester's grading on purpose - kept as in the reference)."""
        if not self.connected:
            return "disconnected"
        if self.rtt < 10:
            return "excellent"
        if self.rtt < 50:
            return "good"
        if self.rtt < 100:
            return "fair"
        return "poor"


@dataclass
class ClusterMetrics:
    timestamp: Optional[_dt.datetime] = jfield("timestamp", time=True)
    total_nodes: int = jfield("total_nodes", default=0)
    healthy_nodes: int = jfield("healthy_nodes", default=0)
    total_pods: int = jfield("total_pods", default=0)
    running_pods: int = jfield("running_pods", default=0)
    total_cpu: int = jfield("total_cpu", default=0)
    used_cpu: int = jfield("used_cpu", default=0)
    cpu_usage_rate: float = jfield("cpu_usage_rate", default=0.0)
    total_memory: int = jfield("total_memory", default=0)
    used_memory: int = jfield("used_memory", default=0)
    memory_usage_rate: float = jfield("memory_usage_rate", default=0.0)
    total_gpus: int = jfield("total_gpus", default=0)
    available_gpus: int = jfield("available_gpus", default=0)
    health_status: str = jfield("health_status", default="")
    issues: Optional[list] = jfield("issues", omitempty=True)


@dataclass
class MetricsSnapshot:
    timestamp: Optional[_dt.datetime] = jfield("timestamp", time=True)
    node_metrics: Optional[dict] = jfield("node_metrics")
    pod_metrics: Optional[dict] = jfield("pod_metrics")
    network_metrics: Optional[list] = jfield("network_metrics")
    cluster_metrics: Optional[ClusterMetrics] = jfield("cluster_metrics")


def any_to_plain(v: Any) -> Any:
    from ..utils.gojson import to_plain

    return to_plain(v)
