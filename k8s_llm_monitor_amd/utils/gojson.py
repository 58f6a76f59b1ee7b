"""Byte-compatible re-implementation of Go ``encoding/json`` output.

The reference server answers every route with ``json.NewEncoder(w).Encode(map[string]interface{}{...})``
(``cmd/server/main.go:175-695``), so API compatibility means reproducing Go's encoder:

* ``map`` keys sorted; struct fields in declaration order (our dataclasses keep field order);
* ``Encode`` appends ``\\n``;
* HTML-safe escaping (``<`` ``>`` ``&`` -> ``\\u003c`` ...), U+2028/2029 escaped, ``\\b``/``\\f``
  short escapes (Go >= 1.22; the reference builds with Go 1.25, ``go.mod:3``);
* ``time.Time`` as RFC 3339 with nanoseconds, trailing zeros trimmed; the zero time
  ``0001-01-01T00:00:00Z``;
* float64 in shortest form, ``'f'`` notation except |x| < 1e-6 or >= 1e21 (``e`` notation with
  ``e-07`` cleaned to ``e-7``);
* nil slices/maps -> ``null``; ``omitempty`` drops false/0/""/nil/empty.

Struct fields are declared with :func:`jfield` (JSON name + omitempty), e.g.
``node_ip: str = jfield("node_ip", omitempty=True)``.
"""
from __future__ import annotations

import dataclasses
import datetime as _dt
import math
from decimal import Decimal
from typing import Any

ZERO_TIME = _dt.datetime(1, 1, 1, tzinfo=_dt.timezone.utc)


class GoTime:
    """Marker for Go's zero ``time.Time`` where a None would be ambiguous."""


def jfield(name: str | None = None, omitempty: bool = False, default=dataclasses.MISSING,
           default_factory=dataclasses.MISSING, time: bool = False):
    """A Go struct field: JSON ``name``, ``omitempty``; ``time=True`` marks a non-pointer
    ``time.Time`` (None encodes as the zero time)."""
    md = {"json": name, "omitempty": omitempty, "time": time}
    if default_factory is not dataclasses.MISSING:
        return dataclasses.field(default_factory=default_factory, metadata=md)
    if default is dataclasses.MISSING:
        default = None
    return dataclasses.field(default=default, metadata=md)


def utcnow() -> _dt.datetime:
    return _dt.datetime.now(_dt.timezone.utc)


def format_time(t: _dt.datetime | None) -> str:
    """RFC3339Nano exactly as Go prints it (microsecond resolution in Python)."""
    if t is None or t == ZERO_TIME:
        return "0001-01-01T00:00:00Z"
    if t.tzinfo is None:
        t = t.replace(tzinfo=_dt.timezone.utc)
    s = t.strftime("%Y-%m-%dT%H:%M:%S")
    if t.microsecond:
        s += ("." + f"{t.microsecond:06d}").rstrip("0")
    off = t.utcoffset()
    if not off:
        return s + "Z"
    mins = int(off.total_seconds()) // 60
    sign = "+" if mins >= 0 else "-"
    mins = abs(mins)
    return f"{s}{sign}{mins // 60:02d}:{mins % 60:02d}"


def format_time_rfc3339(t: _dt.datetime | None) -> str:
    """Go ``time.RFC3339`` (seconds resolution) - used in CRD status fields."""
    if t is None:
        return "0001-01-01T00:00:00Z"
    return format_time(t.replace(microsecond=0))


def parse_time(s: str | None) -> _dt.datetime | None:
    """Parse RFC 3339 (with or without fractional seconds / Z); None on failure."""
    if not s:
        return None
    try:
        x = s.strip()
        if x.endswith("Z"):
            x = x[:-1] + "+00:00"
        if "." in x:  # trim nanoseconds to microseconds for fromisoformat
            head, rest = x.split(".", 1)
            frac = ""
            i = 0
            while i < len(rest) and rest[i].isdigit():
                frac += rest[i]
                i += 1
            x = head + "." + (frac[:6].ljust(6, "0")) + rest[i:]
        t = _dt.datetime.fromisoformat(x)
        if t.tzinfo is None:
            t = t.replace(tzinfo=_dt.timezone.utc)
        if t.year == 1 and t.month == 1 and t.day == 1:
            return ZERO_TIME
        return t
    except ValueError:
        return None


def format_float(f: float) -> str:
    if math.isnan(f) or math.isinf(f):
        return "null"  # Go refuses to encode these (UnsupportedValueError); never crash a handler
    if f == 0:
        return "-0" if math.copysign(1.0, f) < 0 else "0"
    a = abs(f)
    if a < 1e-6 or a >= 1e21:
        r = repr(f)  # shortest round-trip, exponent form in this range
        mant, exp = r.split("e")
        sign = exp[0]
        digits = exp[1:].lstrip("0") or "0"
        if len(digits) < 2:
            digits = "0" + digits
        out = f"{mant}e{sign}{digits}"
        if out[-4] == "e" and out[-3] == "-" and out[-2] == "0":  # Go's e-09 -> e-9 cleanup
            out = out[:-2] + out[-1]
        return out
    r = repr(f)
    if "e" not in r:  # repr is already fixed-point here ([1e-4, 1e16)): Go's digits, maybe a ".0"
        return r.rstrip("0").rstrip(".") if "." in r else r
    s = format(Decimal(r), "f")
    if "." in s:
        s = s.rstrip("0").rstrip(".")
    return s


_json_str = __import__("json").encoder.encode_basestring  # C-accelerated, non-ASCII kept raw

_ESC = {'"': '\\"', "\\": "\\\\", "\n": "\\n", "\r": "\\r", "\t": "\\t", "\b": "\\b", "\f": "\\f",
        "<": "\\u003c", ">": "\\u003e", "&": "\\u0026", "\u2028": "\\u2028", "\u2029": "\\u2029"}


def quote(s: str) -> str:
    r"""Go encoding/json string literal.  Fast path: the C json encoder already produces Go's
    escapes for quotes, backslashes, \n \r \t \b \f and the other control characters
    (\u00xx, lowercase); Go additionally escapes < > & and U+2028 / U+2029.  Strings holding
    lone surrogates (not valid UTF-8; Go writes U+FFFD) take the per-character path."""
    if not s.isascii():
        try:
            s.encode("utf-8")
        except UnicodeEncodeError:
            return _quote_slow(s)
    out = _json_str(s)
    if "<" in out or ">" in out or "&" in out:
        out = out.replace("<", "\\u003c").replace(">", "\\u003e").replace("&", "\\u0026")
    if "\u2028" in out or "\u2029" in out:
        out = out.replace("\u2028", "\\u2028").replace("\u2029", "\\u2029")
    return out


def _quote_slow(s: str) -> str:
    out = ['"']
    for ch in s:
        e = _ESC.get(ch)
        if e is not None:
            out.append(e)
        elif ch < " ":
            out.append("\\u%04x" % ord(ch))
        elif 0xD800 <= ord(ch) <= 0xDFFF:
            out.append("\\ufffd")
        else:
            out.append(ch)
    out.append('"')
    return "".join(out)


def _empty(v: Any) -> bool:
    if v is None or v is False:
        return True
    if isinstance(v, (int, float)) and not isinstance(v, bool) and v == 0:
        return True
    if isinstance(v, (str, list, tuple, dict)) and len(v) == 0:
        return True
    return False


_FIELDS: dict = {}


def _fields(cls) -> list:
    """Per dataclass type, once: (attribute, encoded '"name":', omitempty, time) of every encoded field."""
    fs = _FIELDS.get(cls)
    if fs is None:
        fs = []
        for f in dataclasses.fields(cls):
            md = f.metadata
            if md.get("skip"):
                continue
            fs.append((f.name, quote(md.get("json") or f.name) + ":", bool(md.get("omitempty")), bool(md.get("time"))))
        _FIELDS[cls] = fs
    return fs


def _enc(o: Any, out: list) -> None:
    if o is None:
        out.append("null")
    elif o is True:
        out.append("true")
    elif o is False:
        out.append("false")
    elif isinstance(o, int):
        out.append(str(int(o)))
    elif isinstance(o, float):
        out.append(format_float(o))
    elif isinstance(o, str):
        out.append(quote(o))
    elif isinstance(o, _dt.datetime):
        out.append(quote(format_time(o)))
    elif o is GoTime or isinstance(o, GoTime):
        out.append('"0001-01-01T00:00:00Z"')
    elif dataclasses.is_dataclass(o) and not isinstance(o, type):
        out.append("{")
        first = True
        for attr, key, omitempty, is_time in _fields(type(o)):
            v = getattr(o, attr)
            if omitempty and _empty(v):
                continue
            if is_time and v is None:
                v = ZERO_TIME
            if not first:
                out.append(",")
            first = False
            out.append(key)
            _enc(v, out)
        out.append("}")
    elif isinstance(o, dict):
        out.append("{")
        for i, k in enumerate(sorted(o, key=lambda x: str(x))):
            if i:
                out.append(",")
            out.append(quote(str(k)))
            out.append(":")
            _enc(o[k], out)
        out.append("}")
    elif isinstance(o, (list, tuple)):
        out.append("[")
        for i, v in enumerate(o):
            if i:
                out.append(",")
            _enc(v, out)
        out.append("]")
    elif hasattr(o, "to_go_json"):
        _enc(o.to_go_json(), out)
    else:
        raise TypeError(f"gojson: cannot encode {type(o).__name__}")


def dumps(o: Any) -> str:
    """``json.Marshal`` equivalent (no trailing newline)."""
    out: list = []
    _enc(o, out)
    return "".join(out)


def encode(o: Any) -> bytes:
    """``json.NewEncoder(w).Encode(o)`` equivalent: compact JSON + newline, UTF-8."""
    return (dumps(o) + "\n").encode("utf-8")


def to_plain(o: Any) -> Any:
    """Round-trip through the Go encoding into plain Python values (dicts/lists/str/num)."""
    import json

    return json.loads(dumps(o))
