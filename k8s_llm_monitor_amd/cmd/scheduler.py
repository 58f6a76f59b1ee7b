"""``scheduler`` binary (cmd/scheduler/main.go:20-67): ``-config``, ``-interval`` (default 15s);
in-cluster service account first, then the kubeconfig."""
from __future__ import annotations

import argparse
import logging
import signal
import sys
import threading

from ..monitor.config import ConfigError, load
from ..monitor.uav.agent import parse_go_duration
from ..utils.logsetup import setup_logging


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(prog="scheduler")
    ap.add_argument("-config", "--config", default="./configs/config.yaml")
    ap.add_argument("-interval", "--interval", default="15s", help="reconcile interval (Go duration)")
    ap.add_argument("-max-heartbeat-age", "--max-heartbeat-age", default="0s",
                    help="skip UAVs whose last_update is older (0 = never, the reference behaviour)")
    a = ap.parse_args(argv)
    try:
        cfg = load(a.config)
    except ConfigError as e:
        print(f"load config failed: {e}", file=sys.stderr)
        return 1
    setup_logging(cfg.logging.level, cfg.logging.format, cfg.logging.output)
    from ..monitor.app import make_backend
    from ..monitor.scheduler.controller import SchedulerController

    if (cfg.k8s.backend or "auto") == "auto":
        cfg.k8s.backend = "kube"
    backend = make_backend(cfg)
    ctl = SchedulerController(backend, parse_go_duration(a.interval), parse_go_duration(a.max_heartbeat_age))
    stop = threading.Event()
    signal.signal(signal.SIGINT, lambda *_: stop.set())
    signal.signal(signal.SIGTERM, lambda *_: stop.set())
    ctl.run(stop)
    return 0


if __name__ == "__main__":
    sys.exit(main())
