#!/usr/bin/env bash
# UAV telemetry collection checks against a RUNNING server (reference scripts/test_uav_collection.sh):
# agent pods (when kubectl is available), /api/v1/metrics/uav, per-node lookup (pushed report and
# the first listed node), field integrity (uav_id/gps/battery/flight/health), the low-battery
# (<20%), GPS (<10 satellites) and health (system_status != OK) monitors, the 10-GET latency
# acceptance (<1 s good, 1-3 s fair, >3 s slow = fail), the UAVMetric CRD listing and a per-UAV
# report (tools/smoke.py uav).
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
