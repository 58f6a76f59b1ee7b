"""Deterministic, scenario-driven in-memory Kubernetes cluster with fault injection.

The reference has no fake K8s API at all (its "mock K8s" is simply the absence of
a cluster; multi-node tests need k3d).  This backend serves raw Kubernetes JSON for every resource
the monitor reads or writes - nodes, pods, services, events, network policies, metrics.k8s.io,
CRDs and custom resources (UAVMetric, SchedulingRequest) - plus:

* ``exec``  simulates ``ping -c N -W T <ip>`` / ``curl ... -w %{time_total}`` inside pods with a
  node-to-node latency model (busybox/iputils output format, so the RTT parser is exercised);
* ``http_request`` routes ``http://<podIP>:9090/...`` to an in-process MAVLink simulator for every
  UAV agent pod (the same AgentAPI the real agent serves);
* ``watch`` streams ADDED/MODIFIED/DELETED with resourceVersions (initial synthetic ADDED events
  when started without a resourceVersion, like the API server);
* fault toggles (SURVEY.md §5 "fault-injectable FakeCluster"): node NotReady / pressure, pod
  CrashLoopBackOff / Pending / Failed, metrics-server down, UAV agent unreachable, CoreDNS down,
  network partitions, packet loss and latency, and deny NetworkPolicies;
* ``tick(dt)`` advances simulated time: usage random walks, crash-loop restarts + events, UAV
  physics.

Default topology mirrors the reference's k3d dev cluster (``docs/k3d-deployment.md``;
``deployments/uav-simulator.yaml``: nodes k3d-k8s-llm-monitor-{server-0,agent-0,agent-1}, UAVs at
85/75/90 % battery in AUTO/LOITER/AUTO).  ``FakeCluster.build(n_nodes=..., pods_per_node=...)``
scales it up for benchmarks.
"""
from __future__ import annotations

import copy
import datetime as _dt
import itertools
import random
import re
import threading
import time
import uuid
from typing import Iterator, Optional
from urllib.parse import urlparse

from ...utils.gojson import format_time, utcnow
from ..uav.agent_api import AgentAPI
from ..uav.simulator import MAVLinkSimulator
from .backend import (CRDS, EVENTS, KINDS, NAMESPACES, NETWORK_POLICIES, NODE_METRICS, NODES, POD_METRICS, PODS,
                      SCHEDULING_REQUESTS, SERVICES, UAV_METRICS, GVR, ApiError, ClusterBackend, ExecError,
                      match_fields, match_labels)

K8S_VERSION = {"major": "1", "minor": "31", "gitVersion": "v1.31.5+k3s1", "platform": "linux/amd64"}
GIB = 1 << 30
MIB = 1 << 20


def _ts(t: _dt.datetime) -> str:
    return t.replace(microsecond=0).strftime("%Y-%m-%dT%H:%M:%SZ")


class FakeCluster(ClusterBackend):
    def __init__(self, seed: int = 0):
        self.rng = random.Random(seed)
        self.seed = seed
        self._lock = threading.RLock()
        self._cv = threading.Condition(self._lock)
        self._store: dict[GVR, dict[tuple, dict]] = {}
        self._rv = itertools.count(1000)
        self._log: list[tuple[int, GVR, str, dict]] = []  # (rv, gvr, type, obj) for watches
        self.node_usage: dict[str, tuple[float, float]] = {}  # node -> (cpu cores, mem bytes) baseline
        self.pod_usage: dict[tuple, dict[str, tuple[float, float]]] = {}  # (ns, pod) -> container usage
        self.uav: dict[tuple, tuple[MAVLinkSimulator, AgentAPI]] = {}  # (ns, pod) -> agent
        self.faults = {"metrics_down": False, "agent_down": set(), "partition": set(), "loss": 0.0,
                       "extra_latency_ms": 0.0, "no_ping": set(), "api_down": False}
        self.node_latency_ms: dict[frozenset, float] = {}
        self.now = utcnow().replace(microsecond=0)
        self.sim_time = 0.0
        self.exec_log: list[tuple[str, str, list]] = []
        self._ip = itertools.count(10)

    # ================================================================== construction
    @classmethod
    def build(cls, scenario: str = "k3d", seed: int = 0, n_nodes: int = 3, pods_per_node: int = 4,
              uav_agents: bool = True) -> "FakeCluster":
        fc = cls(seed)
        fc._install_crds()
        for ns in ("default", "kube-system", "monitoring"):
            fc._put(NAMESPACES, {"apiVersion": "v1", "kind": "Namespace",
                                 "metadata": {"name": ns, "uid": str(uuid.UUID(int=fc.rng.getrandbits(128)))},
                                 "status": {"phase": "Active"}})
        if scenario == "k3d" and n_nodes == 3:
            names = ["k3d-k8s-llm-monitor-server-0", "k3d-k8s-llm-monitor-agent-0", "k3d-k8s-llm-monitor-agent-1"]
        else:
            names = [f"node-{i:03d}" for i in range(n_nodes)]
        for i, n in enumerate(names):
            fc.add_node(n, cpu_cores=8 if i else 4, mem_gib=32 if i else 16, control_plane=(i == 0))
        # kube-system
        fc.add_pod("kube-system", "coredns-7b98449c4-x2k5n", names[0], app="kube-dns", image="rancher/mirrored-coredns-coredns:1.11.3",
                   labels={"k8s-app": "kube-dns"}, cpu=(0.1, None), mem=(70 * MIB, 170 * MIB))
        fc.add_pod("kube-system", "metrics-server-5985cbc9d7-jq8bf", names[0], app="metrics-server",
                   image="rancher/mirrored-metrics-server:v0.7.2", cpu=(0.1, None), mem=(70 * MIB, None))
        fc.add_pod("kube-system", "local-path-provisioner-5cf85fd84d-b6gkm", names[0], app="local-path-provisioner",
                   image="rancher/local-path-provisioner:v0.0.30")
        fc.add_service("kube-system", "kube-dns", {"k8s-app": "kube-dns"}, [("dns", 53, "UDP"), ("dns-tcp", 53, "TCP")],
                       cluster_ip="10.43.0.10")
        # default namespace workloads
        web_node = names[1 % len(names)]
        fc.add_pod("default", "nginx-web-6d4cf56db6-8v2mz", web_node, app="nginx", image="nginx:1.25",
                   cpu=(0.1, 0.5), mem=(64 * MIB, 256 * MIB), ports=[80])
        fc.add_pod("default", "busybox-test", names[2 % len(names)], app="busybox", image="busybox:1.36",
                   cpu=(0.05, 0.2), mem=(16 * MIB, 64 * MIB))
        fc.add_pod("default", "frontend-5c7d8f9b4-kq2lp", names[0], app="frontend", image="node:20-alpine",
                   cpu=(0.25, 1.0), mem=(128 * MIB, 512 * MIB), ports=[3000])
        fc.add_pod("default", "backend-84d6b7c5f-wx7rt", web_node, app="backend", image="python:3.12-slim",
                   cpu=(0.5, 1.0), mem=(256 * MIB, 1 * GIB), ports=[8000])
        fc.add_pod("default", "redis-0", names[2 % len(names)], app="redis", image="redis:7.2",
                   cpu=(0.1, 0.5), mem=(128 * MIB, 512 * MIB), ports=[6379])
        fc.add_service("default", "nginx-svc", {"app": "nginx"}, [("http", 80, "TCP")])
        fc.add_service("default", "backend", {"app": "backend"}, [("http", 8000, "TCP")])
        fc.add_service("default", "redis", {"app": "redis"}, [("redis", 6379, "TCP")])
        fc.add_service("default", "kubernetes", None, [("https", 443, "TCP")], cluster_ip="10.43.0.1")
        fc.add_network_policy("default", "redis-allow-backend", {"app": "redis"}, ingress_ports=[("TCP", 6379)])
        # extra generic workloads to scale the cluster
        apps = ["api", "worker", "cache", "queue", "auth", "billing", "search", "metrics", "ingest", "report"]
        for i, n in enumerate(names):
            for j in range(max(0, pods_per_node - (2 if i < 3 else 0))):
                app = apps[(i + j) % len(apps)]
                fc.add_pod("default" if j % 2 == 0 else "monitoring", f"{app}-{fc._suffix()}", n, app=app,
                           image=f"registry.local/{app}:1.{j}", cpu=(0.2, 1.0), mem=(128 * MIB, 512 * MIB))
        if uav_agents:
            presets = [(85.0, "AUTO"), (75.0, "LOITER"), (90.0, "AUTO")]
            for i, n in enumerate(names):
                batt, mode = presets[i % 3]
                fc.add_uav_agent(n, battery=batt, mode=mode)
        for i, a in enumerate(names):
            for j, b in enumerate(names):
                if i < j:
                    fc.node_latency_ms[frozenset((a, b))] = 0.25 + 0.05 * (i + j)
        fc._event("default", "Pod", "nginx-web-6d4cf56db6-8v2mz", "Normal", "Started", "Started container nginx", "kubelet")
        return fc

    def _suffix(self) -> str:
        a = "".join(self.rng.choice("bcdfghjklmnpqrstvwxz2456789") for _ in range(10))
        b = "".join(self.rng.choice("bcdfghjklmnpqrstvwxz2456789") for _ in range(5))
        return f"{a[:9]}-{b}"

    def _next_ip(self, prefix: str) -> str:
        n = next(self._ip)
        return f"{prefix}.{n // 250}.{n % 250 + 2}"

    def _meta(self, name: str, namespace: Optional[str] = None, labels: Optional[dict] = None) -> dict:
        m = {"name": name, "uid": str(uuid.UUID(int=self.rng.getrandbits(128))),
             "creationTimestamp": _ts(self.now - _dt.timedelta(hours=self.rng.randint(1, 96)))}
        if namespace is not None:
            m["namespace"] = namespace
        if labels:
            m["labels"] = dict(labels)
        return m

    def add_node(self, name: str, cpu_cores: int = 8, mem_gib: int = 32, control_plane: bool = False) -> dict:
        labels = {"kubernetes.io/hostname": name, "kubernetes.io/os": "linux", "kubernetes.io/arch": "amd64",
                  "beta.kubernetes.io/instance-type": "k3s"}
        if control_plane:
            labels["node-role.kubernetes.io/control-plane"] = "true"
            labels["node-role.kubernetes.io/master"] = "true"
        disk = 100 * GIB
        node = {"apiVersion": "v1", "kind": "Node", "metadata": self._meta(name, None, labels),
                "spec": {"podCIDR": f"10.42.{len(self._objs(NODES))}.0/24"},
                "status": {"capacity": {"cpu": str(cpu_cores), "memory": f"{mem_gib * 1024 * 1024}Ki",
                                        "ephemeral-storage": f"{disk // 1024}Ki", "pods": "110"},
                           "allocatable": {"cpu": str(cpu_cores), "memory": f"{mem_gib * 1024 * 1024}Ki",
                                           "ephemeral-storage": str(int(disk * 0.93)), "pods": "110"},
                           "conditions": self._node_conditions(),
                           "addresses": [{"type": "InternalIP", "address": f"172.18.0.{len(self._objs(NODES)) + 2}"},
                                         {"type": "Hostname", "address": name}],
                           "nodeInfo": {"kubeletVersion": K8S_VERSION["gitVersion"], "osImage": "K3s v1.31.5+k3s1",
                                        "containerRuntimeVersion": "containerd://1.7.23-k3s2"}}}
        self._put(NODES, node)
        self.node_usage[name] = (cpu_cores * self.rng.uniform(0.1, 0.45), mem_gib * GIB * self.rng.uniform(0.2, 0.55))
        return node

    def _node_conditions(self, ready: bool = True, pressure: Optional[str] = None) -> list:
        ts = _ts(self.now)
        conds = []
        for t in ("MemoryPressure", "DiskPressure", "PIDPressure"):
            on = pressure == t
            conds.append({"type": t, "status": "True" if on else "False", "lastHeartbeatTime": ts,
                          "lastTransitionTime": ts, "reason": f"Kubelet{'Has' if on else 'HasNo'}{t}",
                          "message": f"kubelet has {'insufficient' if on else 'sufficient'} "
                                     f"{t.replace('Pressure', '').lower()} available"})
        conds.append({"type": "Ready", "status": "True" if ready else "Unknown", "lastHeartbeatTime": ts,
                      "lastTransitionTime": ts, "reason": "KubeletReady" if ready else "NodeStatusUnknown",
                      "message": "kubelet is posting ready status" if ready else "Kubelet stopped posting node status."})
        return conds

    def add_pod(self, namespace: str, name: str, node: str, app: str = "", image: str = "busybox:1.36",
                labels: Optional[dict] = None, cpu: tuple = (0.1, None), mem: tuple = (64 * MIB, None),
                ports: Optional[list] = None, phase: str = "Running", env: Optional[dict] = None,
                containers: int = 1) -> dict:
        lbl = {"app": app} if app else {}
        lbl.update(labels or {})
        cs, st = [], []
        for c in range(containers):
            cname = (app or name.split("-")[0]) + (f"-{c}" if c else "")
            res: dict = {}
            if cpu[0] or mem[0]:
                res["requests"] = {}
                if cpu[0]:
                    res["requests"]["cpu"] = f"{int(cpu[0] * 1000)}m"
                if mem[0]:
                    res["requests"]["memory"] = f"{mem[0] // MIB}Mi"
            if cpu[1] or mem[1]:
                res["limits"] = {}
                if cpu[1]:
                    res["limits"]["cpu"] = f"{int(cpu[1] * 1000)}m"
                if mem[1]:
                    res["limits"]["memory"] = f"{mem[1] // MIB}Mi"
            spec_c = {"name": cname, "image": image, "resources": res,
                      "env": [{"name": k, "value": v} for k, v in (env or {"LOG_LEVEL": "info"}).items()]}
            if ports:
                spec_c["ports"] = [{"containerPort": p, "protocol": "TCP"} for p in ports]
            cs.append(spec_c)
            st.append({"name": cname, "image": image, "ready": phase == "Running", "restartCount": 0,
                       "state": {"running": {"startedAt": _ts(self.now - _dt.timedelta(hours=2))}}
                       if phase == "Running" else {"waiting": {"reason": "ContainerCreating"}}})
        ip = self._next_ip("10.42") if phase in ("Running", "Failed") else ""
        started = self.now - _dt.timedelta(minutes=self.rng.randint(5, 3000))
        pod = {"apiVersion": "v1", "kind": "Pod", "metadata": self._meta(name, namespace, lbl),
               "spec": {"nodeName": node if phase != "Pending" else "", "containers": cs,
                        "restartPolicy": "Always", "serviceAccountName": "default"},
               "status": {"phase": phase, "podIP": ip, "hostIP": self._node_ip(node),
                          "startTime": _ts(started) if phase != "Pending" else None,
                          "conditions": [{"type": "Ready", "status": "True" if phase == "Running" else "False"},
                                         {"type": "PodScheduled", "status": "True" if phase != "Pending" else "False"}],
                          "containerStatuses": st}}
        if pod["status"]["startTime"] is None:
            del pod["status"]["startTime"]
        if phase == "Pending":
            pod["status"]["conditions"][1]["reason"] = "Unschedulable"
            pod["status"]["conditions"][1]["message"] = "0/3 nodes are available: insufficient memory."
        self._put(PODS, pod)
        self.pod_usage[(namespace, name)] = {
            c["name"]: ((cpu[0] or 0.05) * self.rng.uniform(0.3, 1.4), (mem[0] or 32 * MIB) * self.rng.uniform(0.5, 1.3))
            for c in cs} if phase == "Running" else {}
        return pod

    def _node_ip(self, node: str) -> str:
        n = self._store.get(NODES, {}).get((None, node))
        if not n:
            return ""
        for a in n["status"].get("addresses", []):
            if a["type"] == "InternalIP":
                return a["address"]
        return ""

    def add_service(self, namespace: str, name: str, selector: Optional[dict], ports: list,
                    cluster_ip: Optional[str] = None, svc_type: str = "ClusterIP") -> dict:
        svc = {"apiVersion": "v1", "kind": "Service", "metadata": self._meta(name, namespace),
               "spec": {"type": svc_type, "clusterIP": cluster_ip or self._next_ip("10.43"),
                        "ports": [{"name": n, "port": p, "protocol": pr, "targetPort": p} for n, p, pr in ports]}}
        if selector:
            svc["spec"]["selector"] = dict(selector)
        self._put(SERVICES, svc)
        return svc

    def add_network_policy(self, namespace: str, name: str, pod_selector: dict, ingress_ports: Optional[list] = None,
                           egress_ports: Optional[list] = None, deny_all: bool = False) -> dict:
        spec: dict = {"podSelector": {"matchLabels": dict(pod_selector)}, "policyTypes": ["Ingress"]}
        if deny_all:
            spec["ingress"] = []
        elif ingress_ports is not None:
            spec["ingress"] = [{"ports": [{"protocol": pr, "port": p} for pr, p in ingress_ports],
                                "from": [{"podSelector": {"matchLabels": {"app": "backend"}}}]}]
        if egress_ports is not None:
            spec["policyTypes"].append("Egress")
            spec["egress"] = [{"ports": [{"protocol": pr, "port": p} for pr, p in egress_ports]}]
        np_ = {"apiVersion": "networking.k8s.io/v1", "kind": "NetworkPolicy", "metadata": self._meta(name, namespace),
               "spec": spec}
        self._put(NETWORK_POLICIES, np_)
        return np_

    def add_uav_agent(self, node: str, battery: float = 100.0, mode: str = "STABILIZE", namespace: str = "default",
                      armed: Optional[bool] = None) -> str:
        name = f"uav-agent-{self._suffix()[:5]}"
        self.add_pod(namespace, name, node, app="uav-agent", image="k8s-uav-agent:dev", cpu=(0.05, 0.2),
                     mem=(32 * MIB, 128 * MIB), ports=[9090], env={"NODE_NAME": node, "REPORT_INTERVAL": "10s"})
        uav_id = f"UAV-{node}"
        sim = MAVLinkSimulator(uav_id, node, seed=self.rng.getrandbits(32), battery_percent=battery, flight_mode=mode,
                               armed=(mode == "AUTO") if armed is None else armed)
        pod = self._store[PODS][(namespace, name)]
        self.uav[(namespace, name)] = (sim, AgentAPI(sim, uav_id, node, pod["status"]["podIP"]))
        return name

    def _install_crds(self) -> None:
        for group, kind, plural, short, status_sub in (("monitoring.io", "UAVMetric", "uavmetrics", "uav", False),
                                                        ("scheduler.io", "SchedulingRequest", "schedulingrequests",
                                                         "sreq", True)):
            ver = {"name": "v1", "served": True, "storage": True,
                   "schema": {"openAPIV3Schema": {"type": "object", "x-kubernetes-preserve-unknown-fields": True}}}
            if status_sub:
                ver["subresources"] = {"status": {}}
            self._put(CRDS, {"apiVersion": "apiextensions.k8s.io/v1", "kind": "CustomResourceDefinition",
                             "metadata": self._meta(f"{plural}.{group}"),
                             "spec": {"group": group, "scope": "Namespaced", "versions": [ver],
                                      "names": {"kind": kind, "plural": plural, "singular": kind.lower(),
                                                "shortNames": [short]}},
                             "status": {"conditions": [{"type": "NamesAccepted", "status": "True"},
                                                       {"type": "Established", "status": "True"}],
                                        "storedVersions": ["v1"]}})

    def _event(self, namespace: str, kind: str, name: str, etype: str, reason: str, message: str,
               component: str, count: int = 1) -> None:
        ev = {"apiVersion": "v1", "kind": "Event",
              "metadata": self._meta(f"{name}.{uuid.UUID(int=self.rng.getrandbits(128)).hex[:16]}", namespace),
              "involvedObject": {"kind": kind, "name": name, "namespace": namespace},
              "reason": reason, "message": message, "type": etype, "count": count,
              "source": {"component": component}, "firstTimestamp": _ts(self.now), "lastTimestamp": _ts(self.now)}
        self._put(EVENTS, ev)

    # ================================================================== storage
    def _objs(self, gvr: GVR) -> dict:
        return self._store.setdefault(gvr, {})

    @staticmethod
    def _key(gvr: GVR, obj: dict) -> tuple:
        md = obj.get("metadata", {})
        return (md.get("namespace") if gvr.namespaced else None, md.get("name"))

    def _put(self, gvr: GVR, obj: dict, etype: Optional[str] = None) -> dict:
        with self._cv:
            key = self._key(gvr, obj)
            store = self._objs(gvr)
            existed = key in store
            rv = next(self._rv)
            obj = copy.deepcopy(obj)
            md = obj.setdefault("metadata", {})
            md["resourceVersion"] = str(rv)
            md.setdefault("creationTimestamp", _ts(self.now))
            md.setdefault("uid", str(uuid.UUID(int=self.rng.getrandbits(128))))
            obj.setdefault("apiVersion", gvr.api_version)
            obj.setdefault("kind", KINDS.get(gvr, "Object"))
            store[key] = obj
            self._log.append((rv, gvr, etype or ("MODIFIED" if existed else "ADDED"), copy.deepcopy(obj)))
            if len(self._log) > 20000:
                del self._log[:10000]
            self._cv.notify_all()
            return copy.deepcopy(obj)

    def _check_api(self) -> None:
        if self.faults["api_down"]:
            raise OSError("dial tcp 127.0.0.1:6443: connect: connection refused")

    # ================================================================== ClusterBackend
    def server_version(self) -> dict:
        self._check_api()
        return dict(K8S_VERSION)

    def list(self, gvr: GVR, namespace: Optional[str] = None, label_selector: str = "",
             field_selector: str = "", limit: int = 0) -> list[dict]:
        self._check_api()
        if gvr in (NODE_METRICS, POD_METRICS):
            return self._metrics_list(gvr, namespace)
        with self._lock:
            out = []
            for (ns, _), obj in sorted(self._objs(gvr).items(), key=lambda kv: (kv[0][0] or "", kv[0][1])):
                if gvr.namespaced and namespace and ns != namespace:
                    continue
                if label_selector and not match_labels(label_selector, obj.get("metadata", {}).get("labels")):
                    continue
                if field_selector and not match_fields(field_selector, obj):
                    continue
                out.append(copy.deepcopy(obj))
                if limit and len(out) >= limit:
                    break
            return out

    def get(self, gvr: GVR, name: str, namespace: Optional[str] = None) -> dict:
        self._check_api()
        if gvr in (NODE_METRICS, POD_METRICS):
            for o in self._metrics_list(gvr, namespace):
                if o["metadata"]["name"] == name:
                    return o
            raise ApiError(404, "NotFound", f'{gvr.resource}.metrics.k8s.io "{name}" not found')
        with self._lock:
            obj = self._objs(gvr).get((namespace if gvr.namespaced else None, name))
            if obj is None:
                res = gvr.resource + (f".{gvr.group}" if gvr.group else "")
                raise ApiError(404, "NotFound", f'{res} "{name}" not found')
            return copy.deepcopy(obj)

    def create(self, gvr: GVR, obj: dict, namespace: Optional[str] = None) -> dict:
        self._check_api()
        with self._lock:
            obj = copy.deepcopy(obj)
            md = obj.setdefault("metadata", {})
            if gvr.namespaced:
                md["namespace"] = namespace or md.get("namespace") or "default"
            if not md.get("name"):
                if md.get("generateName"):
                    md["name"] = md["generateName"] + self._suffix()[:5]
                else:
                    raise ApiError(422, "Invalid", "metadata.name: Required value")
            if self._key(gvr, obj) in self._objs(gvr):
                res = gvr.resource + (f".{gvr.group}" if gvr.group else "")
                raise ApiError(409, "AlreadyExists", f'{res} "{md["name"]}" already exists')
            md["generation"] = 1
            md["creationTimestamp"] = _ts(self.now)
            md["managedFields"] = [{"manager": "k8s-llm-monitor", "operation": "Update", "time": _ts(self.now)}]
            return self._put(gvr, obj, "ADDED")

    def _replace(self, gvr: GVR, obj: dict, namespace: Optional[str], status_only: bool) -> dict:
        self._check_api()
        with self._lock:
            obj = copy.deepcopy(obj)
            md = obj.setdefault("metadata", {})
            if gvr.namespaced:
                md["namespace"] = namespace or md.get("namespace") or "default"
            key = self._key(gvr, obj)
            cur = self._objs(gvr).get(key)
            if cur is None:
                res = gvr.resource + (f".{gvr.group}" if gvr.group else "")
                raise ApiError(404, "NotFound", f'{res} "{md.get("name")}" not found')
            rv = md.get("resourceVersion")
            if rv and rv != cur["metadata"]["resourceVersion"]:
                raise ApiError(409, "Conflict", f'Operation cannot be fulfilled on {gvr.resource} "{md["name"]}": '
                                                "the object has been modified; please apply your changes to the "
                                                "latest version and try again")
            new = copy.deepcopy(cur)
            if status_only:
                new["status"] = obj.get("status")
            else:
                crd_status_sub = gvr == SCHEDULING_REQUESTS  # CRDs with a status subresource ignore status here
                for k, v in obj.items():
                    if k == "status" and crd_status_sub:
                        continue
                    new[k] = v
                if new.get("spec") != cur.get("spec"):
                    new["metadata"]["generation"] = int(cur["metadata"].get("generation", 1)) + 1
            new["metadata"]["managedFields"] = [{"manager": "k8s-llm-monitor", "operation": "Update",
                                                 "time": _ts(self.now)}]
            return self._put(gvr, new, "MODIFIED")

    def update(self, gvr: GVR, obj: dict, namespace: Optional[str] = None) -> dict:
        return self._replace(gvr, obj, namespace, status_only=False)

    def update_status(self, gvr: GVR, obj: dict, namespace: Optional[str] = None) -> dict:
        if gvr == UAV_METRICS:  # no status subresource on this CRD (deployments/uav-metrics-crd.yaml)
            raise ApiError(404, "NotFound", "the server could not find the requested resource")
        return self._replace(gvr, obj, namespace, status_only=True)

    def delete(self, gvr: GVR, name: str, namespace: Optional[str] = None) -> None:
        self._check_api()
        with self._cv:
            key = (namespace if gvr.namespaced else None, name)
            obj = self._objs(gvr).pop(key, None)
            if obj is None:
                raise ApiError(404, "NotFound", f'{gvr.resource} "{name}" not found')
            rv = next(self._rv)
            obj["metadata"]["resourceVersion"] = str(rv)
            self._log.append((rv, gvr, "DELETED", obj))
            self._cv.notify_all()
        self.pod_usage.pop((namespace, name), None) if gvr == PODS else None
        if gvr == PODS and (namespace, name) in self.uav:
            self.uav.pop((namespace, name))[0].stop()

    def watch(self, gvr: GVR, namespace: Optional[str] = None, resource_version: str = "",
              timeout_s: float = 300.0, stop=None) -> Iterator[tuple[str, dict]]:
        self._check_api()
        deadline = time.monotonic() + timeout_s
        with self._lock:
            if resource_version:
                rv = int(resource_version)
                if self._log and rv < self._log[0][0] - 1:
                    yield "ERROR", {"kind": "Status", "code": 410, "reason": "Expired",
                                    "message": "too old resource version"}
                    return
            else:
                rv = self._log[-1][0] if self._log else 0
                initial = [o for (ns, _), o in self._objs(gvr).items() if not (gvr.namespaced and namespace and ns != namespace)]
        if not resource_version:
            for o in initial:
                yield "ADDED", copy.deepcopy(o)
        while True:
            with self._cv:
                pending = [e for e in self._log if e[0] > rv and e[1] == gvr]
                if not pending:
                    remaining = deadline - time.monotonic()
                    if remaining <= 0 or (stop is not None and stop.is_set()):
                        return
                    self._cv.wait(min(0.2, remaining))
                    continue
            for erv, _, etype, obj in pending:
                rv = erv
                if gvr.namespaced and namespace and obj.get("metadata", {}).get("namespace") != namespace:
                    continue
                yield etype, copy.deepcopy(obj)
            if stop is not None and stop.is_set():
                return

    def pod_logs(self, namespace: str, pod: str, tail_lines: int = 100) -> str:
        p = self.get(PODS, pod, namespace)
        app = p["metadata"].get("labels", {}).get("app", pod)
        restarts = sum(c.get("restartCount", 0) for c in p["status"].get("containerStatuses", []))
        lines = [f"{format_time(self.now)} INFO {app} started, listening"]
        if restarts:
            lines += [f"{format_time(self.now)} ERROR {app}: panic: runtime error: invalid memory address",
                      f"{format_time(self.now)} FATAL {app} exited with code 2"]
        return "\n".join(lines[-tail_lines:]) + "\n"

    # ------------------------------------------------------------------ metrics.k8s.io
    def _metrics_list(self, gvr: GVR, namespace: Optional[str]) -> list[dict]:
        if self.faults["metrics_down"]:
            raise ApiError(503, "ServiceUnavailable", "the server is currently unable to handle the request "
                                                      f"(get {gvr.resource}.metrics.k8s.io)")
        out = []
        with self._lock:
            if gvr == NODE_METRICS:
                for (_, name), node in sorted(self._objs(NODES).items(), key=lambda kv: kv[0][1]):
                    ready = any(c["type"] == "Ready" and c["status"] == "True" for c in node["status"]["conditions"])
                    if not ready:
                        continue  # metrics-server drops nodes it cannot scrape
                    cpu, mem = self.node_usage.get(name, (0.0, 0.0))
                    for (ns, pn), cu in self.pod_usage.items():
                        pod = self._objs(PODS).get((ns, pn))
                        if pod and pod["spec"].get("nodeName") == name:
                            cpu += sum(u[0] for u in cu.values())
                            mem += sum(u[1] for u in cu.values())
                    out.append({"apiVersion": "metrics.k8s.io/v1beta1", "kind": "NodeMetrics",
                                "metadata": {"name": name, "creationTimestamp": _ts(self.now)},
                                "timestamp": _ts(self.now), "window": "20s",
                                "usage": {"cpu": f"{int(cpu * 1e9)}n", "memory": f"{int(mem // 1024)}Ki"}})
            else:
                for (ns, pn), pod in sorted(self._objs(PODS).items(), key=lambda kv: (kv[0][0], kv[0][1])):
                    if namespace and ns != namespace:
                        continue
                    cu = self.pod_usage.get((ns, pn))
                    if not cu or pod["status"].get("phase") != "Running":
                        continue
                    out.append({"apiVersion": "metrics.k8s.io/v1beta1", "kind": "PodMetrics",
                                "metadata": {"name": pn, "namespace": ns, "creationTimestamp": _ts(self.now)},
                                "timestamp": _ts(self.now), "window": "15s",
                                "containers": [{"name": c, "usage": {"cpu": f"{int(u[0] * 1e9)}n",
                                                                     "memory": f"{int(u[1] // 1024)}Ki"}}
                                               for c, u in cu.items()]})
        return out

    # ------------------------------------------------------------------ exec (ping / curl)
    def _pod_by_ip(self, ip: str) -> Optional[dict]:
        for pod in self._objs(PODS).values():
            if pod["status"].get("podIP") == ip:
                return pod
        return None

    def _blocked_by_policy(self, target: dict) -> bool:
        labels = target["metadata"].get("labels", {})
        for np_ in self._objs(NETWORK_POLICIES).values():
            if np_["metadata"].get("namespace") != target["metadata"]["namespace"]:
                continue
            sel = np_["spec"].get("podSelector", {}).get("matchLabels", {})
            if all(labels.get(k) == v for k, v in sel.items()) and np_["spec"].get("ingress") == []:
                return True
        return False

    def _path_rtt(self, src: dict, dst: dict) -> Optional[float]:
        a, b = src["spec"].get("nodeName"), dst["spec"].get("nodeName")
        if dst["status"].get("phase") != "Running" or self._blocked_by_policy(dst):
            return None
        if frozenset((a, b)) in self.faults["partition"]:
            return None
        for n in (a, b):
            node = self._objs(NODES).get((None, n))
            if node and not any(c["type"] == "Ready" and c["status"] == "True" for c in node["status"]["conditions"]):
                return None
        base = 0.05 if a == b else self.node_latency_ms.get(frozenset((a, b)), 0.4)
        return base + self.faults["extra_latency_ms"]

    def exec(self, namespace: str, pod: str, container: str, command: list[str],
             timeout_s: float = 30.0) -> tuple[str, str]:
        self._check_api()
        src = self.get(PODS, pod, namespace)
        self.exec_log.append((namespace, pod, list(command)))
        if src["status"].get("phase") != "Running":
            raise ExecError(f"unable to upgrade connection: container not found (\"{container}\")")
        cmd = command[-1] if command[:2] == ["sh", "-c"] else " ".join(command)
        image = src["spec"]["containers"][0]["image"]
        m = re.match(r"ping\s+-c\s+(\d+)\s+-W\s+(\d+)\s+(\S+)", cmd)
        if m:
            if (namespace, pod) in self.faults["no_ping"] or "distroless" in image:
                raise ExecError('command terminated with exit code 127, stderr: sh: ping: not found')
            n, ip = int(m.group(1)), m.group(3)
            dst = self._pod_by_ip(ip)
            rtt = self._path_rtt(src, dst) if dst else None
            lines = [f"PING {ip} ({ip}): 56 data bytes"]
            got = []
            for i in range(n):
                lost = rtt is None or self.rng.random() < self.faults["loss"]
                if not lost:
                    t = rtt * self.rng.uniform(0.8, 1.3)
                    got.append(t)
                    lines.append(f"64 bytes from {ip}: seq={i} ttl=62 time={t:.3f} ms")
            loss = int(round(100 * (n - len(got)) / n))
            lines += ["", f"--- {ip} ping statistics ---",
                      f"{n} packets transmitted, {len(got)} packets received, {loss}% packet loss"]
            if got:
                lines.append(f"round-trip min/avg/max = {min(got):.3f}/{sum(got) / len(got):.3f}/{max(got):.3f} ms")
            out = "\n".join(lines) + "\n"
            if not got:
                raise ExecError(f"command terminated with exit code 1, stderr: ")
            return out, ""
        m = re.match(r"curl\s+.*?(?:-m\s+(\d+)\s+)?http://([^:/\s]+):(\d+)", cmd)
        if m and cmd.startswith("curl"):
            if "busybox" in image or "distroless" in image:
                raise ExecError("command terminated with exit code 127, stderr: sh: curl: not found")
            ip = m.group(2)
            dst = self._pod_by_ip(ip)
            rtt = self._path_rtt(src, dst) if dst else None
            if rtt is None:
                return "0.000000", ""  # curl -w prints time_total even on connect failure
            return f"{(rtt * 3 + 0.4) / 1000.0:.6f}", ""
        raise ExecError(f"command terminated with exit code 127, stderr: sh: {cmd.split()[0]}: not found")

    # ------------------------------------------------------------------ in-cluster HTTP (UAV agents)
    def http_request(self, method: str, url: str, body: Optional[bytes] = None,
                     timeout_s: float = 5.0) -> tuple[int, bytes]:
        u = urlparse(url)
        with self._lock:
            target = None
            for (ns, pn), (sim, api) in self.uav.items():
                pod = self._objs(PODS).get((ns, pn))
                if pod and pod["status"].get("podIP") == u.hostname and u.port == 9090:
                    target = (pod, api)
                    break
        if target is None:
            raise OSError(f"dial tcp {u.hostname}:{u.port}: connect: no route to host")
        pod, api = target
        if pod["spec"].get("nodeName") in self.faults["agent_down"] or pod["status"].get("phase") != "Running":
            raise TimeoutError(f"Get \"{url}\": context deadline exceeded (Client.Timeout exceeded while awaiting headers)")
        code, _, data = api.handle(method, u.path, body)
        return code, data

    # ================================================================== faults
    def _mutate(self, gvr: GVR, name: str, namespace: Optional[str], fn) -> dict:
        with self._lock:
            obj = copy.deepcopy(self._objs(gvr)[(namespace if gvr.namespaced else None, name)])
            fn(obj)
            return self._put(gvr, obj, "MODIFIED")

    def set_node_ready(self, node: str, ready: bool) -> None:
        def f(o):
            o["status"]["conditions"] = self._node_conditions(ready=ready)
        self._mutate(NODES, node, None, f)
        if not ready:
            self._event("default", "Node", node, "Normal", "NodeNotReady",
                        f"Node {node} status is now: NodeNotReady", "node-controller")

    def set_node_pressure(self, node: str, pressure: Optional[str]) -> None:
        def f(o):
            o["status"]["conditions"] = self._node_conditions(ready=True, pressure=pressure)
        self._mutate(NODES, node, None, f)
        if pressure:
            self._event("default", "Node", node, "Warning", f"NodeHas{pressure}",
                        f"Node {node} status is now: NodeHas{pressure}", "kubelet")
            if pressure == "MemoryPressure":
                cpu, _ = self.node_usage[node]
                cap = self._mem_capacity(node)
                self.node_usage[node] = (cpu, cap * 0.93)

    def _mem_capacity(self, node: str) -> float:
        from .backend import value
        return float(value(self._objs(NODES)[(None, node)]["status"]["capacity"]["memory"]))

    def set_node_cpu_load(self, node: str, fraction: float) -> None:
        from .backend import parse_quantity
        cap = parse_quantity(self._objs(NODES)[(None, node)]["status"]["capacity"]["cpu"])
        _, mem = self.node_usage[node]
        self.node_usage[node] = (cap * fraction, mem)

    def crashloop_pod(self, namespace: str, name: str, restarts: int = 12) -> None:
        def f(o):
            o["status"]["phase"] = "Running"
            o["status"]["conditions"][0]["status"] = "False"
            for cs in o["status"]["containerStatuses"]:
                cs["ready"] = False
                cs["restartCount"] = restarts
                cs["state"] = {"waiting": {"reason": "CrashLoopBackOff",
                                           "message": f"back-off 5m0s restarting failed container={cs['name']}"}}
                cs["lastState"] = {"terminated": {"exitCode": 2, "reason": "Error"}}
        self._mutate(PODS, name, namespace, f)
        self._event(namespace, "Pod", name, "Warning", "BackOff", "Back-off restarting failed container", "kubelet",
                    count=restarts)

    def fail_pod(self, namespace: str, name: str, reason: str = "Error") -> None:
        def f(o):
            o["status"]["phase"] = "Failed"
            o["status"]["reason"] = reason
            o["status"]["conditions"][0]["status"] = "False"
            for cs in o["status"]["containerStatuses"]:
                cs["ready"] = False
                cs["state"] = {"terminated": {"exitCode": 137, "reason": reason}}
        self._mutate(PODS, name, namespace, f)
        self.pod_usage[(namespace, name)] = {}
        self._event(namespace, "Pod", name, "Warning", reason, f"Container terminated: {reason}", "kubelet")

    def overload_pod(self, namespace: str, name: str, fraction_of_limit: float = 0.97) -> None:
        """Drive a pod's memory (and cpu) usage to ``fraction_of_limit`` of its limits."""
        from .backend import parse_quantity
        pod = self._objs(PODS)[(namespace, name)]
        cu = {}
        for c in pod["spec"]["containers"]:
            lim = c.get("resources", {}).get("limits", {})
            cu[c["name"]] = (parse_quantity(lim.get("cpu", "1")) * fraction_of_limit,
                             parse_quantity(lim.get("memory", "512Mi")) * fraction_of_limit)
        self.pod_usage[(namespace, name)] = cu
        self._event(namespace, "Pod", name, "Warning", "OOMKilling", "Memory usage near the container limit",
                    "kubelet")

    def set_coredns(self, running: bool) -> None:
        for (ns, pn) in list(self._objs(PODS)):
            if ns == "kube-system" and "coredns" in pn:
                if running:
                    self._mutate(PODS, pn, ns, lambda o: o["status"].update(phase="Running"))
                else:
                    self.crashloop_pod(ns, pn, restarts=7)
                    self._mutate(PODS, pn, ns, lambda o: o["status"].update(phase="Pending"))

    def deny_ingress(self, namespace: str, selector: dict, name: str = "deny-all-ingress") -> None:
        self.add_network_policy(namespace, name, selector, deny_all=True)

    def partition(self, node_a: str, node_b: str, on: bool = True) -> None:
        key = frozenset((node_a, node_b))
        (self.faults["partition"].add if on else self.faults["partition"].discard)(key)

    def find_pods(self, namespace: Optional[str] = None, app: Optional[str] = None) -> list[str]:
        with self._lock:
            return [pn for (ns, pn), p in sorted(self._objs(PODS).items())
                    if (namespace is None or ns == namespace)
                    and (app is None or p["metadata"].get("labels", {}).get("app") == app)]

    # ================================================================== time
    def tick(self, dt: float = 10.0) -> None:
        """Advance simulated time: usage random walk, crash-loop restarts, UAV physics."""
        with self._lock:
            self.sim_time += dt
            self.now = self.now + _dt.timedelta(seconds=dt)
            for n, (c, m) in list(self.node_usage.items()):
                self.node_usage[n] = (max(0.0, c * self.rng.uniform(0.95, 1.05)), max(0.0, m * self.rng.uniform(0.98, 1.02)))
            for k, cu in self.pod_usage.items():
                self.pod_usage[k] = {c: (u[0] * self.rng.uniform(0.9, 1.1), u[1] * self.rng.uniform(0.99, 1.01))
                                     for c, u in cu.items()}
            crash = [(ns, pn) for (ns, pn), p in self._objs(PODS).items()
                     if any(cs.get("state", {}).get("waiting", {}).get("reason") == "CrashLoopBackOff"
                            for cs in p["status"].get("containerStatuses", []))]
        for ns, pn in crash:
            def f(o):
                for cs in o["status"]["containerStatuses"]:
                    cs["restartCount"] += 1
            self._mutate(PODS, pn, ns, f)
        for sim, _ in list(self.uav.values()):
            sim.step(min(dt, 5.0))
