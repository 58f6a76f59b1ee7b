#!/usr/bin/env bash
# Start the monitor server on a config (default: the FakeCluster dev config, no GPU needed), run
# the HTTP smoke suite against it, stop it.  Mirrors the reference's test_server.sh /
# test_with_mock_k8s.sh (health, cluster status, 400 on a bad body, pod-communication, query).
#   scripts/test_server.sh [config.yaml] [port]
set -u
cd "$(dirname "$0")/.."
CONFIG="${1:-configs/config.dev.yaml}"
PORT="${2:-${SERVER_PORT:-8080}}"
export SERVER_PORT="$PORT"
python -m k8s_llm_monitor_amd.cmd.server -config "$CONFIG" &
PID=$!
trap 'kill "$PID" 2>/dev/null; wait "$PID" 2>/dev/null' EXIT
python tools/smoke.py all --url "http://127.0.0.1:${PORT}" --wait 60
RC=$?
echo "smoke exit status: $RC"
exit $RC
