#!/usr/bin/env bash
# Checks a RUNNING server's console and REST endpoints (reference test_web_interface.sh).
#   SERVER_URL=http://127.0.0.1:8080 scripts/test_web_interface.sh
set -u
cd "$(dirname "$0")/.."
URL="${SERVER_URL:-http://127.0.0.1:8080}"
if ! python tools/smoke.py server --url "$URL" --no-query; then
  echo "web interface checks failed against $URL"
  exit 1
fi
echo "console: open $URL in a browser (auto-refreshes every 15 s)"
