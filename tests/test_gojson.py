"""Go encoding/json compatibility."""
import datetime as dt
from dataclasses import dataclass

from k8s_llm_monitor_amd.utils import gojson
from k8s_llm_monitor_amd.utils.gojson import format_float, format_time, jfield, parse_time, quote
from k8s_llm_monitor_amd.monitor.types import NetworkMetrics, PodInfo, UAVReport


def test_floats_like_strconv():
    cases = {100.0: "100", 0.1: "0.1", 1e-7: "1e-7", 1.5e-7: "1.5e-7", 1e21: "1e+21", 1e20: "100000000000000000000",
             0.000001: "0.000001", 123456789.0: "123456789", -2.5: "-2.5", 1e-10: "1e-10", 0.9: "0.9", 0.0: "0",
             40.78: "40.78", 2.0 / 3.0: "0.6666666666666666"}
    for f, s in cases.items():
        assert format_float(f) == s, (f, format_float(f))


def test_string_escaping_is_html_safe():
    assert quote("<a&b>") == '"\\u003ca\\u0026b\\u003e"'
    assert quote("x y ") == '"x\\u2028y\\u2029"'
    assert quote("\x01\b\f\n\r\t\"\\") == '"\\u0001\\b\\f\\n\\r\\t\\"\\\\"'
    assert quote("中文 ok") == '"中文 ok"'


def test_time_rfc3339nano():
    t = dt.datetime(2025, 10, 11, 10, 0, 0, 123450, tzinfo=dt.timezone.utc)
    assert format_time(t) == "2025-10-11T10:00:00.12345Z"
    assert format_time(t.replace(microsecond=0)) == "2025-10-11T10:00:00Z"
    assert format_time(None) == "0001-01-01T00:00:00Z"
    tz8 = dt.timezone(dt.timedelta(hours=8))
    assert format_time(dt.datetime(2025, 1, 2, 3, 4, 5, tzinfo=tz8)) == "2025-01-02T03:04:05+08:00"
    assert parse_time("2025-10-11T10:00:00.123456789Z") == dt.datetime(2025, 10, 11, 10, 0, 0, 123456,
                                                                         tzinfo=dt.timezone.utc)


def test_maps_sorted_structs_ordered_newline():
    out = gojson.encode({"b": 1, "a": [1, 2], "c": None, "d": {}})
    assert out == b'{"a":[1,2],"b":1,"c":null,"d":{}}\n'

    @dataclass
    class S:
        z: int = jfield("z", default=1)
        a: str = jfield("a", omitempty=True, default="")
        t: object = jfield("t", time=True)

    assert gojson.dumps(S()) == '{"z":1,"t":"0001-01-01T00:00:00Z"}'


def test_model_nil_vs_empty_and_omitempty():
    p = PodInfo(name="x")
    d = gojson.to_plain(p)
    assert d["labels"] is None and d["containers"] is None
    assert list(d) == ["name", "namespace", "status", "node_name", "ip", "labels", "start_time", "containers"]
    nm = gojson.to_plain(NetworkMetrics(source_pod="a", target_pod="b"))
    assert "error" not in nm and "bandwidth_mbps" not in nm and nm["rtt_ms"] == 0
    r = gojson.to_plain(UAVReport(node_name="n"))
    assert set(r) == {"node_name", "uav_id", "source", "status", "timestamp"}


def test_uav_report_roundtrip():
    d = {"node_name": "n1", "uav_id": "U", "source": "agent", "status": "active", "timestamp": "2025-01-01T00:00:00Z",
         "heartbeat_interval_seconds": 10, "state": {"uav_id": "U", "battery": {"remaining_percent": 55.5},
                                                     "health": {"messages": ["a"]}}, "metadata": {"agent": "x"},
         "unknown": 1}
    r = UAVReport.from_dict(d)
    assert r.state.battery.remaining_percent == 55.5 and r.state.health.messages == ["a"]
    back = gojson.to_plain(r)
    assert back["state"]["battery"]["remaining_percent"] == 55.5 and back["heartbeat_interval_seconds"] == 10


def test_quote_fast_path_matches_per_character_encoder():
    """quote()'s C-accelerated path produces exactly the per-character Go encoder's output."""
    import random

    from k8s_llm_monitor_amd.utils import gojson

    alphabet = ['"', "\\", "\n", "\r", "\t", "\b", "\f", "<", ">", "&", " ", "\x00", "\x01", "\x1f", "\x7f",
                "a", "\u96c6", "\u00e9", "\U0001f600", "\ud800", "\udfff", "/", "'", "\u0085", "\ufeff", "\u2028", "\u2029"]
    rng = random.Random(0)
    for _ in range(5000):
        s = "".join(rng.choice(alphabet) for _ in range(rng.randint(0, 24)))
        assert gojson.quote(s) == gojson._quote_slow(s), repr(s)
