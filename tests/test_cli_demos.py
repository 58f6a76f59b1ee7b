"""The test-k8s smoke CLI (B4, cmd/test-k8s/main.go:44-185) and the five demos (B5-B9,
cmd/demos/*) run end to end against the in-memory FakeCluster."""
from __future__ import annotations

import pytest

from k8s_llm_monitor_amd.cmd import demos, test_k8s


def test_test_k8s_cli_watches_and_analyses(capsys):
    assert test_k8s.main(["--fake", "--watch-seconds", "1.0"]) == 0
    out = capsys.readouterr().out
    assert "== connection:" in out and "== cluster info:" in out
    assert "== analysis" in out
    # the watch really runs (the reference's returns at once): the injected crash loop is seen
    watched = [ln for ln in out.splitlines() if ln.startswith("== watched:")]
    assert watched and "pods=0" not in watched[0]


@pytest.mark.parametrize("demo,needle", [
    ("debug", "step 2 cluster info:"),
    ("network", "->"),
    ("rtt", "avg="),
    ("crd", "CRD "),
    ("live", "pods:"),
])
def test_demos_run_on_fake_cluster(demo, needle, capsys):
    assert demos.main([demo, "--fake", "--seconds", "0.6"]) == 0
    assert needle in capsys.readouterr().out
