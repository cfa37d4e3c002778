"""Server-log beautifier: a stdin filter (reference ``cmd/utils/log-beautifier/main.go``).

* lines without ``{`` are echoed; JSON is parsed from the first ``{`` so
  ``docker compose logs`` prefixes are tolerated (``main.go:27-44``);
* ``server starting`` → SETUP ✓ ``Server Listening (addr=…)``;
  ``gRPC call received`` → CONNECTION ✓ ``gRPC Connection (method)`` then a pending
  ``○ method`` line under EXECUTION; ``gRPC call finished`` → ✓/✗ (✗ when ``code != "OK"``)
  with the duration measured by the filter's own clock, erasing the pending line with
  ``\\033[1A\\033[K``; ``server shutting down`` / ``server stopped`` → SHUTDOWN ✓
  (``processServerLogEntry``, ``main.go:47-83``).

Difference: pending calls are keyed by ``request_id`` when the log line carries one (our
interceptor adds it), so concurrent calls of one method no longer collide.
"""
from __future__ import annotations

import json
import sys
import time
from typing import IO, Dict, Iterable, Optional

from ..utils.slog import go_duration
from .jest import BOLD, GRAY, GREEN, RED, RESET

ERASE_LINE = "\033[1A\033[K"


class Beautifier:
    def __init__(self, out: Optional[IO[str]] = None, clock=time.monotonic):
        self.out = out or sys.stdout
        self.current_suite = ""
        self.pending: Dict[str, float] = {}
        self.clock = clock

    def _header(self, name: str) -> None:
        if self.current_suite != name:
            sep = "─" * 10
            self.out.write(f"\n{GRAY}{sep} {BOLD}{name} {sep}{RESET}\n")
            self.current_suite = name

    def _step(self, status: str, message: str, details: str = "") -> None:
        color, symbol = (GREEN, "✓") if status == "PASS" else (RED, "✗")
        if status in ("PASS", "FAIL"):
            self.out.write(ERASE_LINE)
        if details:
            self.out.write(f"  {color}{symbol}{RESET} {message} {GRAY}({details}){RESET}\n")
        else:
            self.out.write(f"  {color}{symbol}{RESET} {message}\n")

    def feed(self, line: str) -> None:
        line = line.rstrip("\n")
        start = line.find("{")
        if start < 0:
            self.out.write(line + "\n")
            return
        try:
            e = json.loads(line[start:])
        except ValueError:
            self.out.write(line + "\n")
            return
        if isinstance(e, dict):
            self.entry(e)

    def entry(self, e: dict) -> None:
        msg = e.get("msg", "") if isinstance(e.get("msg"), str) else ""
        method = e.get("method", "") if isinstance(e.get("method"), str) else ""
        key = str(e["request_id"]) if "request_id" in e else method
        if msg == "server starting":
            self._header("SETUP")
            self._step("PASS", "Server Listening", f"addr={e.get('address')}")
        elif msg == "gRPC call received":
            self._header("CONNECTION")
            self._step("PASS", "gRPC Connection", method)
            self._header("EXECUTION")
            self.pending[key] = self.clock()
            self.out.write(f"  ○ {GRAY}{method}\n")
        elif msg == "gRPC call finished":
            t0 = self.pending.pop(key, None)
            if t0 is None:
                return
            dur = go_duration(round(self.clock() - t0, 3))
            code = e.get("code", "")
            self._step("PASS" if code == "OK" else "FAIL", method, dur)
        elif msg in ("server shutting down", "server stopped"):
            self._header("SHUTDOWN")
            self._step("PASS", msg)

    def run(self, lines: Iterable[str]) -> None:
        for line in lines:
            self.feed(line)
            try:
                self.out.flush()
            except Exception:
                pass


def main(argv=None) -> int:
    """``docker compose logs -f | python -m polykey_service_amd.report.log_beautifier``"""
    Beautifier().run(sys.stdin)
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
