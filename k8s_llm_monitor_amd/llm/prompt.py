"""Prompt construction for the diagnostic LLM.

``build_cluster_context`` follows the reference's ``prepareLLMContext``
(``docs/metrics-usage-example.md:244-288``) line for line: the cluster overview, one line per
node with ``[资源压力]`` / ``[不健康]`` flags, and the "problem pods" (not Running, not Ready,
restarts > 5, or near a limit).  Additions the analysis engine uses when the data exists: recent
Warning events (bounded by ``analysis.max_context_events``, config.go:94), network-probe
failures and UAV health.  Nodes and pods are emitted sorted (Go map iteration is random; a
deterministic prompt makes answers reproducible and lets identical questions share a prefix).

``build_query_prompt`` wraps it exactly like ``analyzewithLLM`` (:295-301).  The context is cut
to ``token_budget`` tokens (middle-out, keeping the overview and the question) so a huge cluster
cannot exceed the model's context.
"""
from __future__ import annotations

from typing import Callable, Optional

from ..monitor.types import MetricsSnapshot

SYSTEM_PREAMBLE = ("You are a Kubernetes site-reliability assistant. Answer using only the cluster "
                   "data provided; name the affected nodes/pods and give concrete next steps.\n")


def build_cluster_context(snap: MetricsSnapshot, events: Optional[list] = None, uavs: Optional[dict] = None,
                          max_events: int = 100) -> str:
    c = snap.cluster_metrics
    lines = ["", "集群状态概览:",
             f"- 健康状态: {c.health_status if c else 'unknown'}",
             f"- 节点: {c.total_nodes if c else 0}个 (健康: {c.healthy_nodes if c else 0}个)",
             f"- Pod: {c.total_pods if c else 0}个 (运行中: {c.running_pods if c else 0}个)",
             f"- CPU使用率: {(c.cpu_usage_rate if c else 0.0):.1f}%",
             f"- 内存使用率: {(c.memory_usage_rate if c else 0.0):.1f}%",
             "", "节点详情:"]
    for name in sorted(snap.node_metrics or {}):
        n = snap.node_metrics[name]
        s = f"- {name}: CPU={n.cpu_usage_rate:.1f}%, MEM={n.memory_usage_rate:.1f}%"
        if n.is_under_pressure():
            s += " [资源压力]"
        if not n.healthy:
            s += " [不健康]"
        lines.append(s)
    lines += ["", "问题Pod:"]
    for key in sorted(snap.pod_metrics or {}):
        p = snap.pod_metrics[key]
        if p.phase != "Running" or not p.ready or p.restarts > 5:
            lines.append(f"- {key}: 状态={p.phase}, 就绪={'true' if p.ready else 'false'}, 重启={p.restarts}次")
        if p.is_over_limit():
            lines.append(f"- {key}: 资源使用接近限制")
    if c and c.issues:
        lines += ["", "集群问题:"] + [f"- {i}" for i in c.issues]
    bad_net = [m for m in snap.network_metrics or [] if not m.connected or m.rtt >= 50]
    if bad_net:
        lines += ["", "网络探测异常:"]
        for m in bad_net:
            lines.append(f"- {m.source_pod} -> {m.target_pod}: "
                         + (f"不通 ({m.error})" if not m.connected else f"RTT={m.rtt:.2f}ms ({m.get_quality()})"))
    if events:
        warn = [e for e in events if getattr(e, "type", "") == "Warning"][-max_events:]
        if warn:
            lines += ["", "最近告警事件:"]
            for e in warn:
                lines.append(f"- [{e.reason}] {e.message} (x{e.count})")
    if uavs:
        bad = []
        for node in sorted(uavs):
            st = uavs[node].get("state") if isinstance(uavs[node], dict) else None
            status = uavs[node].get("status") if isinstance(uavs[node], dict) else ""
            if st is None:
                continue
            if status == "stale" or st.health.system_status != "OK" or st.battery.remaining_percent < 20:
                bad.append(f"- {node}: UAV {st.uav_id} 电量={st.battery.remaining_percent:.1f}%, "
                           f"状态={st.health.system_status}, 模式={st.flight.mode}"
                           + (", 心跳超时" if status == "stale" else ""))
        if bad:
            lines += ["", "UAV异常:"] + bad
    return "\n".join(lines) + "\n"


def build_query_prompt(context: str, question: str) -> str:
    return f"\n基于以下Kubernetes集群指标数据:\n\n{context}\n\n请回答用户问题: {question}\n"


def build_pod_communication_prompt(analysis, pod_facts: str, rtt_summary: str = "") -> str:
    issues = "\n".join(f"- {i}" for i in analysis.issues or []) or "- (none)"
    sols = "\n".join(f"- {s}" for s in analysis.solutions or []) or "- (none)"
    return (f"\nPod通信诊断: {analysis.pod_a} -> {analysis.pod_b}\n规则检查结论: {analysis.status} "
            f"(置信度 {analysis.confidence})\n\n发现的问题:\n{issues}\n\n建议:\n{sols}\n\nPod信息:\n{pod_facts}\n"
            f"{rtt_summary}\n请解释最可能的根因，并按优先级给出排查步骤。\n")


def build_analysis_prompt(kind: str, context: str, params: Optional[dict] = None) -> str:
    params = params or {}
    if kind == "anomaly_detection":
        task = "请找出上述集群指标中的异常 (资源压力、重启、不健康节点、网络与UAV异常)，按严重程度排序。"
    elif kind == "root_cause":
        target = params.get("target") or params.get("pod") or params.get("node") or "集群"
        symptom = params.get("symptom") or params.get("question") or ""
        task = f"请针对 {target} 进行根因分析{('，症状: ' + symptom) if symptom else ''}，给出证据链和修复建议。"
    else:
        task = params.get("question") or "请总结集群健康状况。"
    return f"\n基于以下Kubernetes集群指标数据:\n\n{context}\n\n{task}\n"


def trim_to_budget(text: str, encode: Callable[[str], list], budget: int) -> str:
    """Keep the head (overview) and tail; drop whole lines from the middle until it fits."""
    if budget <= 0 or len(encode(text)) <= budget:
        return text
    lines = text.split("\n")
    head, tail = lines[:12], lines[12:]
    while tail and len(encode("\n".join(head + ["- ... (truncated)"] + tail))) > budget:
        tail = tail[max(1, len(tail) // 8):]
    return "\n".join(head + ["- ... (truncated)"] + tail)
