"""Synthetic cluster-state prompts for benchmarks (no real cluster or dataset is reachable).

The text follows the reference's prompt sketch ``prepareLLMContext`` / ``analyzewithLLM``
(``docs/metrics-usage-example.md:244-306``): a cluster overview, per-node CPU/MEM lines with the
[资源压力]/[不健康] flags, the "problem pods" list, then the user question.  The production path
builds the same text from a live metrics snapshot (``llm/prompt.py``); this module fabricates a
snapshot-shaped text directly so the benchmark can size prompts without a cluster.
"""
from __future__ import annotations

import random

QUESTIONS = [
    "为什么我的pod频繁重启？",
    "Which nodes are under resource pressure and what should I do about it?",
    "Why is pod default/api-gateway not ready?",
    "集群内存使用率为什么这么高？",
    "Is the cluster healthy enough to schedule a new batch job?",
    "What is the root cause of the CrashLoopBackOff in namespace kube-system?",
    "Why can't pod default/frontend reach default/backend?",
    "Which pods are close to their memory limits?",
]


def synthetic_cluster_prompt(seed: int, n_nodes: int = 16, n_pods: int = 100, question: str | None = None) -> str:
    ctx, q = synthetic_context(seed, n_nodes, n_pods, question)
    return f"\n基于以下Kubernetes集群指标数据:\n\n{ctx}\n\n请回答用户问题: {q}\n"


def synthetic_context(seed: int, n_nodes: int = 16, n_pods: int = 100, question: str | None = None) -> tuple[str, str]:
    """(cluster-context text, question) - the two parts /api/v1/query combines."""
    r = random.Random(seed)
    healthy = sum(1 for _ in range(n_nodes) if r.random() > 0.1)
    running = int(n_pods * r.uniform(0.8, 0.97))
    cpu = r.uniform(20, 95)
    mem = r.uniform(20, 95)
    status = "critical" if cpu > 90 or mem > 90 else ("warning" if cpu > 80 or mem > 80 else "healthy")
    lines = [
        "",
        "集群状态概览:",
        f"- 健康状态: {status}",
        f"- 节点: {n_nodes}个 (健康: {healthy}个)",
        f"- Pod: {n_pods}个 (运行中: {running}个)",
        f"- CPU使用率: {cpu:.1f}%",
        f"- 内存使用率: {mem:.1f}%",
        "",
        "节点详情:",
    ]
    for i in range(n_nodes):
        c, m = r.uniform(5, 99), r.uniform(5, 99)
        s = f"- node-{i:03d}.cluster.local: CPU={c:.1f}%, MEM={m:.1f}%"
        if c > 80 or m > 80:
            s += " [资源压力]"
        if r.random() < 0.08:
            s += " [不健康]"
        lines.append(s)
    lines += ["", "问题Pod:"]
    apps = ["api-gateway", "frontend", "backend", "redis", "postgres", "kafka", "worker", "scheduler", "nginx",
            "prometheus", "grafana", "coredns", "etcd", "ingress", "auth", "billing"]
    nss = ["default", "kube-system", "monitoring", "prod", "staging"]
    for j in range(n_pods):
        if r.random() < 0.35:
            name = f"{r.choice(nss)}/{r.choice(apps)}-{r.randrange(16**8):08x}-{r.randrange(36**5):05x}"
            phase = r.choice(["Running", "Pending", "Failed", "CrashLoopBackOff", "Running"])
            lines.append(f"- {name}: 状态={phase}, 就绪={str(r.random() < 0.4).lower()}, 重启={r.randrange(0, 40)}次")
            if r.random() < 0.3:
                lines.append(f"- {name}: 资源使用接近限制")
    ctx = "\n".join(lines) + "\n"
    return ctx, question or QUESTIONS[seed % len(QUESTIONS)]
