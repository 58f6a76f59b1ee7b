"""``server`` binary (cmd/server/main.go:23-172).

    python -m k8s_llm_monitor_amd.cmd.server -config ./configs/config.yaml

Multi-GPU (one process per GPU, ``torchrun --nproc-per-node N``):
* ``llm.tp_size = N``   - one tensor-parallel engine; rank 0 serves HTTP, ranks 1.. mirror its steps.
* ``llm.tp_size = 1``   - N data-parallel replicas, replica r serves on ``server.port + r`` (put a
                          Kubernetes Service / load balancer in front, as for any replica set).
Single process, ``llm.dp_replicas = N``: one HTTP server whose queries a least-loaded router spreads
over N engine processes, one per GPU (engine/dp.py).
"""
from __future__ import annotations

import argparse
import logging
import sys

from ..monitor.config import ConfigError, load
from ..utils.logsetup import setup_logging


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(prog="server", prefix_chars="-")
    ap.add_argument("-config", "--config", default="./configs/config.yaml", help="config file path")
    a = ap.parse_args(argv)
    try:
        cfg = load(a.config)
    except ConfigError as e:
        print(f"Failed to load config: {e}", file=sys.stderr)
        return 1
    setup_logging(cfg.logging.level, cfg.logging.format, cfg.logging.output)
    log = logging.getLogger("server")
    pstate = None
    if cfg.llm.provider.lower() in ("local-rocm", "local", "rocm"):
        from ..parallel.state import env_world, init_parallel

        ws, _, _ = env_world()
        if ws > 1:
            pstate = init_parallel(tp_size=cfg.llm.tp_size)
            if pstate.tp_rank != 0:  # TP worker: no HTTP, mirror the leader's engine steps
                from ..engine import LLMEngine
                from ..monitor.app import engine_config

                eng = LLMEngine(engine_config(cfg), pstate=pstate)
                eng.warmup()
                log.info("TP worker rank %d ready", pstate.rank)
                eng.worker_loop()
                return 0
            cfg.server.port += pstate.dp_rank
    from ..monitor.app import build_monitor
    from ..monitor.server import make_server, serve_until_signal

    mon = build_monitor(cfg, pstate=pstate)
    srv = make_server(mon.app, cfg.server.host, cfg.server.port)
    serve_until_signal(srv, on_stop=mon.close)
    return 0


if __name__ == "__main__":
    sys.exit(main())
