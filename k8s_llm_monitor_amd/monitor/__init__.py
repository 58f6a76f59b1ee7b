"""Kubernetes monitoring control plane (API-compatible with Sabre94/k8s-llm-monitor): config,
cluster access, metrics manager, rule analysis, REST server, UAV agent, scheduler controller."""
