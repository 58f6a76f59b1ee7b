#!/usr/bin/env bash
# Development mode, no cluster and no model: the server must still start, answer /health and serve
# the console, answer the cluster routes with the reference's dev-mode warning / 503 bodies
# (cmd/server/main.go:43-51,196-204,234-237,284-293,330-333) and reject bad bodies;
# the rtt demo must fail cleanly (the reference's test_with_mock_k8s.sh checks the same).
#   scripts/test_with_mock_k8s.sh [port]
set -u
cd "$(dirname "$0")/.."
PORT="${1:-8080}"
CFG="$(mktemp --suffix .yaml)"
printf 'server:\n  port: %s\nk8s:\n  backend: "none"\nllm:\n  provider: "none"\nmetrics:\n  enabled: true\n' "$PORT" > "$CFG"
python -m k8s_llm_monitor_amd.cmd.server -config "$CFG" &
PID=$!
trap 'kill "$PID" 2>/dev/null; wait "$PID" 2>/dev/null; rm -f "$CFG"' EXIT
URL="http://127.0.0.1:${PORT}"
for _ in $(seq 1 60); do curl -sf "$URL/health" >/dev/null && break; sleep 0.5; done
FAIL=0
check() {  # name, expected HTTP status, curl args...
  local name="$1" want="$2"; shift 2
  local got
  got=$(curl -s -o /dev/null -w '%{http_code}' "$@")
  if [ "$got" = "$want" ]; then echo "ok   $name ($got)"; else echo "FAIL $name: got $got want $want"; FAIL=1; fi
}
check health 200 "$URL/health"
check console 200 "$URL/"
check cluster-status 200 "$URL/api/v1/cluster/status"
check pods-dev-mode-warning 200 "$URL/api/v1/pods"          # {"status": "warning", "pods": []}
check metrics-unavailable 503 "$URL/api/v1/metrics/cluster"
check pod-comm-unavailable 503 -X POST -d '{not json' "$URL/api/v1/analyze/pod-communication"  # client checked first
check wrong-method 405 -X DELETE "$URL/api/v1/query"
check query-bad-json 400 -X POST -d '{not json' "$URL/api/v1/query"
echo "rtt demo without a cluster (must exit, not hang):"
timeout 10s python -m k8s_llm_monitor_amd.cmd.demos rtt >/dev/null 2>&1
RC=$?
if [ "$RC" = 124 ]; then echo "FAIL rtt demo hung"; FAIL=1; else echo "ok   rtt demo exited ($RC)"; fi
exit $FAIL
