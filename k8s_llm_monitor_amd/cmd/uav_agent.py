"""``uav-agent`` binary (cmd/uav-agent/main.go:22-324)."""
from __future__ import annotations

import argparse
import logging
import os
import signal
import sys
import threading

from ..monitor.uav.agent import UAVAgent, parse_go_duration
from ..utils.logsetup import setup_logging


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(prog="uav-agent")
    ap.add_argument("-port", "--port", type=int, default=9090)
    ap.add_argument("-master-url", "--master-url", default="")
    ap.add_argument("-report-interval", "--report-interval", default="")
    a = ap.parse_args(argv)
    setup_logging("info", "text", "stdout")
    log = logging.getLogger("uav-agent")
    interval = 0.0
    for src in (a.report_interval, os.environ.get("REPORT_INTERVAL", "").strip()):
        if src and interval <= 0:
            try:
                interval = parse_go_duration(src)
            except ValueError as e:
                log.warning("Invalid REPORT_INTERVAL value %r: %s", src, e)
    agent = UAVAgent(os.environ.get("NODE_NAME", ""), os.environ.get("NODE_IP", ""), a.port,
                     a.master_url or os.environ.get("MASTER_URL", ""), interval or 15.0)
    log.info("Starting UAV Agent... UAV ID: %s Node: %s IP: %s Port: %d", agent.uav_id, agent.node_name,
             agent.node_ip, a.port)
    agent.start()
    stop = threading.Event()
    signal.signal(signal.SIGINT, lambda *_: stop.set())
    signal.signal(signal.SIGTERM, lambda *_: stop.set())
    stop.wait()
    log.info("Shutting down UAV agent...")
    agent.stop()
    return 0


if __name__ == "__main__":
    sys.exit(main())
