#!/usr/bin/env bash
# UAV telemetry collection checks against a RUNNING server (reference scripts/test_uav_collection.sh):
# agent pods (when kubectl is available), /api/v1/metrics/uav, per-node lookup after a pushed
# report, battery/GPS fields, and the UAVMetric CRD listing.
#   SERVER_URL=http://127.0.0.1:8081 scripts/test_uav_collection.sh
set -u
cd "$(dirname "$0")/.."
URL="${SERVER_URL:-http://127.0.0.1:8081}"
if command -v kubectl >/dev/null 2>&1; then
  N=$(kubectl get pods -l app=uav-agent --field-selector=status.phase=Running -o name 2>/dev/null | wc -l)
  echo "running uav-agent pods: $N"
  if [ "$N" -eq 0 ]; then
    echo "  (deploy them with: kubectl apply -f deployments/uav-agent-daemonset.yaml)"
  fi
else
  echo "kubectl not found: skipping the agent pod check"
fi
python tools/smoke.py uav --url "$URL"
