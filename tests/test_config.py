import pytest

from k8s_llm_monitor_amd.monitor.config import ConfigError, load, parse_namespaces


def _write(tmp_path, text):
    p = tmp_path / "config.yaml"
    p.write_text(text)
    return str(p)


def test_defaults_match_reference(tmp_path):
    c = load(_write(tmp_path, "{}"))
    assert (c.server.host, c.server.port, c.server.debug) == ("0.0.0.0", 8080, False)
    assert (c.k8s.namespace, c.k8s.watch_namespaces) == ("default", "default")
    assert (c.llm.provider, c.llm.model, c.llm.max_tokens, c.llm.temperature, c.llm.timeout) == ("openai", "gpt-4", 2000, 0.1, 30)
    assert c.storage.type == "memory"
    assert (c.monitoring.metrics_interval, c.monitoring.event_retention, c.monitoring.log_retention) == (30, 168, 24)
    m = c.metrics
    assert (m.enabled, m.collect_interval, m.namespaces, m.enable_node, m.enable_pod, m.enable_network,
            m.enable_custom, m.cache_retention) == (True, 30, ["default"], True, True, False, False, 300)
    assert (c.analysis.enable_prediction, c.analysis.enable_auto_fix, c.analysis.max_context_events) == (True, False, 100)
    assert (c.logging.level, c.logging.format, c.logging.output) == ("info", "json", "stdout")


def test_yaml_then_env_precedence(tmp_path, monkeypatch):
    p = _write(tmp_path, "server:\n  port: 8081\nmetrics:\n  namespaces: [a, b]\nllm:\n  provider: local-rocm\n  tp_size: 8\n")
    monkeypatch.setenv("SERVER_PORT", "9000")
    monkeypatch.setenv("METRICS_ENABLE_NETWORK", "true")
    monkeypatch.setenv("OPENAI_API_KEY", "sk-x")
    monkeypatch.setenv("OPENAI_BASE_URL", "http://llm")
    c = load(p)
    assert c.server.port == 9000
    assert c.metrics.namespaces == ["a", "b"] and c.metrics.enable_network is True
    assert c.llm.provider == "local-rocm" and c.llm.tp_size == 8
    assert c.llm.api_key == "sk-x" and c.llm.base_url == "http://llm"
    monkeypatch.setenv("METRICS_NAMESPACES", "x,y")
    assert load(p).metrics.namespaces == ["x", "y"]


def test_missing_file_and_bad_values(tmp_path):
    with pytest.raises(ConfigError):
        load(str(tmp_path / "nope.yaml"))
    with pytest.raises(ConfigError):
        load(_write(tmp_path, "server:\n  port: notanint\n"))


def test_parse_namespaces():
    assert parse_namespaces("") == ["default"]
    assert parse_namespaces(" a, ,b ") == ["a", "b"]
