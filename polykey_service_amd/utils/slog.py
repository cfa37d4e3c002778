"""Structured logging with Go ``log/slog`` JSON-handler semantics.

The reference logs with ``slog.New(slog.NewJSONHandler(os.Stdout, nil))``
(``cmd/polykey/main.go:55``) and the dev client with a DEBUG-level JSON handler writing
into an in-memory buffer (``cmd/dev_client/main.go:108-111``).  The message strings and
keys are an API: the Jest-style reporters (``test/utils/beautify.go``,
``cmd/utils/log-beautifier/main.go``) parse them.  This module reproduces the line shape
``{"time":..., "level":"INFO", "msg":..., <attrs>}`` and Go's ``time.Duration.String()``
formatting so log consumers written against the reference keep working.
"""
from __future__ import annotations

import datetime as _dt
import io
import json
import sys
import threading
import time as _time
from typing import IO, Any, Optional

DEBUG, INFO, WARN, ERROR = -4, 0, 4, 8
_LEVEL_NAMES = {DEBUG: "DEBUG", INFO: "INFO", WARN: "WARN", ERROR: "ERROR"}
_LEVEL_FROM_NAME = {"debug": DEBUG, "info": INFO, "warn": WARN, "warning": WARN, "error": ERROR}


def level_from_name(name: str, default: int = INFO) -> int:
    return _LEVEL_FROM_NAME.get((name or "").strip().lower(), default)


def go_duration(seconds: float) -> str:
    """Format like Go's ``time.Duration.String()`` (e.g. ``1.5ms``, ``2m3.25s``, ``0s``)."""
    ns = int(round(seconds * 1e9))
    if ns == 0:
        return "0s"
    neg = ns < 0
    ns = abs(ns)
    if ns < 1000:
        out = f"{ns}ns"
    elif ns < 1_000_000:
        out = _frac(ns, 1000) + "µs"
    elif ns < 1_000_000_000:
        out = _frac(ns, 1_000_000) + "ms"
    else:
        h, rem = divmod(ns, 3600 * 1_000_000_000)
        m, rem = divmod(rem, 60 * 1_000_000_000)
        s = _frac(rem, 1_000_000_000) + "s"
        out = (f"{h}h" if h else "") + (f"{m}m" if h or m else "") + s
    return "-" + out if neg else out


def _frac(v: int, unit: int) -> str:
    whole, frac = divmod(v, unit)
    if frac == 0:
        return str(whole)
    width = len(str(unit)) - 1
    return f"{whole}." + f"{frac:0{width}d}".rstrip("0")


def parse_go_duration(text: str) -> float:
    """Parse a Go duration string (``5s``, ``1m30s``, ``250ms``, ``1.5h``) into seconds.

    Raises ``ValueError`` on malformed input, like ``time.ParseDuration``.
    """
    units = {"ns": 1e-9, "us": 1e-6, "µs": 1e-6, "μs": 1e-6, "ms": 1e-3, "s": 1.0, "m": 60.0, "h": 3600.0}
    s = text.strip()
    if not s:
        raise ValueError("time: invalid duration " + repr(text))
    sign = 1.0
    if s[0] in "+-":
        sign = -1.0 if s[0] == "-" else 1.0
        s = s[1:]
    if s == "0":
        return 0.0
    total, i, n = 0.0, 0, len(s)
    if n == 0:
        raise ValueError("time: invalid duration " + repr(text))
    while i < n:
        j = i
        while j < n and (s[j].isdigit() or s[j] == "."):
            j += 1
        if j == i or s[i:j] == ".":
            raise ValueError("time: invalid duration " + repr(text))
        num = float(s[i:j])
        k = j
        while k < n and not (s[k].isdigit() or s[k] == "."):
            k += 1
        unit = s[j:k]
        if unit not in units:
            raise ValueError(("time: missing unit in duration " if not unit else
                              "time: unknown unit " + repr(unit) + " in duration ") + repr(text))
        total += num * units[unit]
        i = k
    return sign * total


_SEC_CACHE: list = [None, "", ""]  # whole second -> its "YYYY-MM-DDTHH:MM:SS" and zone suffix


def _rfc3339nano(ts: Optional[float] = None) -> str:
    """Go's time.RFC3339Nano (trailing zeros of the fraction dropped).  The date/zone part is
    formatted once per second: every RPC logs three records on the serving event loop."""
    t = _time.time() if ts is None else ts
    us = int(round(t * 1e6))
    sec, micro = divmod(us, 1_000_000)
    if _SEC_CACHE[0] != sec:
        now = _dt.datetime.fromtimestamp(sec, _dt.timezone.utc).astimezone()
        off = now.utcoffset() or _dt.timedelta(0)
        if off == _dt.timedelta(0):
            tz = "Z"
        else:
            mins = int(off.total_seconds() // 60)
            sign = "+" if mins >= 0 else "-"
            mins = abs(mins)
            tz = f"{sign}{mins // 60:02d}:{mins % 60:02d}"
        _SEC_CACHE[:] = [sec, now.strftime("%Y-%m-%dT%H:%M:%S"), tz]
    frac = f".{micro:06d}".rstrip("0").rstrip(".")
    return _SEC_CACHE[1] + frac + _SEC_CACHE[2]


def _jsonable(v: Any) -> Any:
    if isinstance(v, (str, int, float, bool)) or v is None:
        return v
    if isinstance(v, (list, tuple)):
        return [_jsonable(x) for x in v]
    if isinstance(v, dict):
        return {str(k): _jsonable(x) for k, x in v.items()}
    if isinstance(v, BaseException):
        return str(v)
    return str(v)


class Logger:
    """Minimal slog-like logger: ``logger.info("msg", key=value, ...)``.

    Attribute order is preserved (Python keeps kwargs order), matching slog's output order.
    """

    def __init__(self, stream: Optional[IO[str]] = None, level: int = INFO, text: bool = False, **base_attrs):
        self.stream = stream if stream is not None else sys.stdout
        self.level = level
        self.text = text
        self.base = base_attrs
        self._lock = threading.Lock()

    def with_attrs(self, **attrs) -> "Logger":
        lg = Logger(self.stream, self.level, self.text, **{**self.base, **attrs})
        lg._lock = self._lock
        return lg

    def enabled(self, level: int) -> bool:
        return level >= self.level

    def log(self, level: int, msg: str, **attrs) -> None:
        if level < self.level:
            return
        rec = {"time": _rfc3339nano(), "level": _LEVEL_NAMES.get(level, str(level)), "msg": msg}
        for k, v in {**self.base, **attrs}.items():
            rec[k] = _jsonable(v)
        if self.text:
            line = " ".join(f"{k}={_text_val(v)}" for k, v in rec.items())
        else:
            line = json.dumps(rec, ensure_ascii=False, separators=(",", ":"))
        with self._lock:
            self.stream.write(line + "\n")
            try:
                self.stream.flush()
            except Exception:
                pass

    def debug(self, msg: str, **a) -> None:
        self.log(DEBUG, msg, **a)

    def info(self, msg: str, **a) -> None:
        self.log(INFO, msg, **a)

    def warn(self, msg: str, **a) -> None:
        self.log(WARN, msg, **a)

    warning = warn

    def error(self, msg: str, **a) -> None:
        self.log(ERROR, msg, **a)


def _text_val(v: Any) -> str:
    s = v if isinstance(v, str) else json.dumps(v)
    return json.dumps(s) if (" " in s or "=" in s or '"' in s) else s


class BufferLogger(Logger):
    """Logger writing into an in-memory buffer (dev client, ``dev_client/main.go:108``)."""

    def __init__(self, level: int = DEBUG):
        super().__init__(io.StringIO(), level)

    def lines(self):
        return self.stream.getvalue().split("\n")


_default = Logger()


def default() -> Logger:
    return _default


def set_default(lg: Logger) -> None:
    global _default
    _default = lg
