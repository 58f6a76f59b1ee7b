#!/usr/bin/env bash
# Build the image, import it into a k3d cluster, roll out the UAV agent DaemonSet and print the
# agents' endpoints (reference scripts/build-and-deploy-uav-agent.sh).  One image serves every
# binary (server / scheduler / uav_agent); the DaemonSet picks the agent entry point.
#   CLUSTER=k8s-llm-monitor IMAGE=k8s-llm-monitor-amd:dev scripts/build-and-deploy-uav-agent.sh
set -euo pipefail
cd "$(dirname "$0")/.."
IMAGE="${IMAGE:-k8s-llm-monitor-amd:dev}"
CLUSTER="${CLUSTER:-k8s-llm-monitor}"
docker build -t "$IMAGE" .
k3d image import "$IMAGE" -c "$CLUSTER"
kubectl apply -f deployments/uav-metrics-crd.yaml
kubectl apply -f deployments/uav-agent-daemonset.yaml
kubectl rollout status daemonset/uav-agent -n default --timeout=120s
kubectl get pods -l app=uav-agent -o wide
kubectl get pods -l app=uav-agent \
  -o custom-columns=NAME:.metadata.name,NODE:.spec.nodeName,IP:.status.podIP,HOST_IP:.status.hostIP --no-headers |
  while read -r name node pod_ip host_ip; do
    echo "  - $name (node $node)"
    echo "    http://$host_ip:9090/health"
    echo "    http://$host_ip:9090/api/v1/state"
  done
