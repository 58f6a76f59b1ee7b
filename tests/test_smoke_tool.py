"""tools/smoke.py (what scripts/*.sh run) against an in-process server on the FakeCluster dev
config: every check of the reference's shell smoke tests must pass."""
import os
import sys
import threading

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))


def test_smoke_suites_pass(tmp_path):
    import smoke

    from k8s_llm_monitor_amd.monitor.app import build_monitor
    from k8s_llm_monitor_amd.monitor.config import load
    from k8s_llm_monitor_amd.monitor.server import make_server

    cfg = load(os.path.join(ROOT, "configs", "config.dev.yaml"))
    mon = build_monitor(cfg)
    srv = make_server(mon.app, "127.0.0.1", 0)
    port = srv.server_address[1]
    th = threading.Thread(target=srv.serve_forever, daemon=True)
    th.start()
    try:
        assert smoke.main(["all", "--url", f"http://127.0.0.1:{port}", "--wait", "10"]) == 0
    finally:
        srv.shutdown()
        mon.close()
