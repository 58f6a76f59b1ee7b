"""Scheduler controller (controller.go) and the UAV simulator / agent API (mavlink_simulator.go)."""
import json

from k8s_llm_monitor_amd.monitor.cluster.backend import SCHEDULING_REQUESTS, UAV_METRICS
from k8s_llm_monitor_amd.monitor.cluster.client import K8sClient
from k8s_llm_monitor_amd.monitor.cluster.fake import FakeCluster
from k8s_llm_monitor_amd.monitor.scheduler.controller import SchedulerController
from k8s_llm_monitor_amd.monitor.types import UAVReport, UAVState
from k8s_llm_monitor_amd.monitor.uav.agent_api import AgentAPI
from k8s_llm_monitor_amd.monitor.uav.simulator import MAVLinkSimulator
from k8s_llm_monitor_amd.utils.gojson import parse_time


def _req(fc, name, workload=("job", "default"), min_batt=0, preferred=None, status=None):
    spec = {"workload": {"name": workload[0], "namespace": workload[1]}}
    if min_batt:
        spec["minBatteryPercent"] = min_batt
    if preferred:
        spec["preferredNodes"] = preferred
    obj = {"apiVersion": "scheduler.io/v1", "kind": "SchedulingRequest", "metadata": {"name": name}, "spec": spec}
    fc.create(SCHEDULING_REQUESTS, obj, "default")
    if status:
        o = fc.get(SCHEDULING_REQUESTS, name, "default")
        o["status"] = status
        fc.update_status(SCHEDULING_REQUESTS, o, "default")


def _uav(client, node, battery, status="active"):
    s = UAVState(uav_id=f"UAV-{node}", node_name=node)
    s.battery.remaining_percent = battery
    client.upsert_uav_metric(UAVReport(node_name=node, uav_id=f"UAV-{node}", status=status, state=s))


def test_assignment_scoring_and_failures():
    fc = FakeCluster.build(seed=1, uav_agents=False)
    c = K8sClient(fc)
    _uav(c, "n1", 80)
    _uav(c, "n2", 75)
    _uav(c, "n3", 99, status="offline")
    _req(fc, "a")
    _req(fc, "b", preferred=["N2"])
    _req(fc, "c", min_batt=90)
    _req(fc, "d", workload=("", "default"))
    _req(fc, "e", status={"phase": "Assigned", "assignedNode": "x"})
    ctl = SchedulerController(fc)
    assert ctl.reconcile() == 4
    st = {o["metadata"]["name"]: o.get("status", {}) for o in fc.list(SCHEDULING_REQUESTS)}
    assert st["a"]["phase"] == "Assigned" and st["a"]["assignedNode"] == "n1" and st["a"]["score"] == 80
    assert st["a"]["message"] == "选中节点 n1 (电量 80.0%)" and st["a"]["assignedUAV"] == "UAV-n1"
    assert st["b"]["assignedNode"] == "n2" and st["b"]["score"] == 85
    assert st["c"] == {"phase": "Failed", "assignedNode": "", "assignedUAV": "", "score": 0, "message": "无满足要求的 UAV 节点",
                       "lastUpdated": st["c"]["lastUpdated"]}
    assert st["d"]["phase"] == "Failed" and st["d"]["message"] == "workload name/namespace 不能为空"
    assert st["e"] == {"phase": "Assigned", "assignedNode": "x"}
    assert parse_time(st["a"]["lastUpdated"]) is not None
    assert ctl.reconcile() == 0  # idempotent: decided requests are skipped


def test_upsert_uav_metric_create_then_update():
    fc = FakeCluster.build(seed=1, uav_agents=False)
    c = K8sClient(fc)
    assert c.upsert_uav_metric(UAVReport(node_name="Edge_Node.1", uav_id="UAV_X", node_ip="10.0.0.1")) == "created"
    o = fc.get(UAV_METRICS, "uavmetric-edge-node-1", "default")
    assert o["metadata"]["labels"]["monitoring.io/uav-id"] == "uav-x"
    assert o["status"]["collection_status"] == "active" and o["spec"] == {"node_name": "Edge_Node.1", "uav_id": "UAV_X"}
    s = UAVState()
    s.battery.remaining_percent = 42.0
    assert c.upsert_uav_metric(UAVReport(node_name="Edge_Node.1", uav_id="UAV_X", state=s)) == "updated"
    o = fc.get(UAV_METRICS, "uavmetric-edge-node-1", "default")
    assert o["spec"]["battery"]["remaining_percent"] == 42.0 and set(o["spec"]) == {"node_name", "uav_id", "gps",
                                                                                     "battery", "flight", "health"}
    crs = c.list_uav_metrics_crd("")
    assert len(crs) == 1 and crs[0].kind == "UAVMetric" and crs[0].group == "monitoring.io"


def test_simulator_physics():
    sim = MAVLinkSimulator("U", "n", seed=0, battery_percent=20.5, flight_mode="AUTO", armed=True)
    sim.step(10.0)  # 100 ticks at 0.1 %/s -> -1 %
    s = sim.get_state()
    assert abs(s.battery.remaining_percent - 19.5) < 1e-6
    assert s.health.system_status == "WARNING" and "Low battery warning" in s.health.messages
    assert abs(s.battery.voltage - (22.2 - 80.5 * 0.04)) < 1e-6
    sim.step(100.0)
    s = sim.get_state()
    assert s.health.system_status == "CRITICAL" and len(s.health.messages) <= 10
    assert abs(s.gps.latitude - 39.9042) < 0.0011
    s.health.messages.append("x")  # a copy: the live state is untouched
    assert "x" not in sim.get_state().health.messages


def test_agent_api_routes():
    sim = MAVLinkSimulator("UAV-n", "n", seed=0)
    api = AgentAPI(sim, "UAV-n", "n", "1.2.3.4")
    code, _, body = api.handle("GET", "/api/v1/state")
    d = json.loads(body)
    assert code == 200 and d["status"] == "success" and d["data"]["uav_id"] == "UAV-n"
    assert api.handle("POST", "/api/v1/state")[0] == 405
    assert json.loads(api.handle("POST", "/api/v1/command/arm")[2])["message"] == "Armed successfully"
    code, _, body = api.handle("POST", "/api/v1/command/takeoff", b"{}")
    assert json.loads(body)["message"] == "Taking off to 50.0m" and sim.get_state().flight.mode == "AUTO"
    assert api.handle("POST", "/api/v1/command/mode", b"not json")[0] == 400
    assert json.loads(api.handle("POST", "/api/v1/command/mode", b'{"mode":"RTL"}')[2])["message"] == "Flight mode set to RTL"
    assert json.loads(api.handle("GET", "/api/v1/battery")[2])["data"]["cell_count"] == 6
    h = json.loads(api.handle("GET", "/health")[2])
    assert h == {**h, "status": "healthy", "uav_id": "UAV-n", "node_ip": "1.2.3.4"}
    assert api.handle("GET", "/nope")[0] == 404


def test_deployment_manifests_parse_and_configmap_current():
    """Every manifest is valid YAML with kind/apiVersion; the simulator ConfigMap embeds the current
    mock_server.py (tools/gen_uav_configmap.py), and every example SchedulingRequest satisfies the
    CRD's required fields."""
    import glob
    import os
    import subprocess
    import sys

    import yaml

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    for path in glob.glob(os.path.join(root, "deployments", "*.yaml")) + glob.glob(os.path.join(root, "examples",
                                                                                                 "*.yaml")):
        with open(path, encoding="utf-8") as f:
            docs = [d for d in yaml.safe_load_all(f) if d]
        assert docs, path
        for d in docs:
            assert d.get("apiVersion") and d.get("kind"), path
            if d["kind"] == "SchedulingRequest":
                w = d["spec"]["workload"]
                assert w["name"] and w["namespace"], path
                assert 0 <= d["spec"].get("minBatteryPercent", 0) <= 100, path
    r = subprocess.run([sys.executable, os.path.join(root, "tools", "gen_uav_configmap.py"), "--check"],
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
