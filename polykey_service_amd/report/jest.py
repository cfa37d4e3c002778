"""Jest-style reporter for newline-delimited JSON logs (reference ``test/utils/beautify.go``).

Two modes, chosen from the first parseable line (``beautify.go:48-57``):

* **app mode** (line has ``msg``) — renders the dev client's log into SETUP / CONNECTION /
  EXECUTION / ERROR suites (``processAppLogEntry``, ``beautify.go:68-112``);
* **test mode** (line has ``Test``/``Action``) — renders ``go test -json``-shaped events
  (``processGoTestEntry``, ``beautify.go:114-139``); :mod:`.pytest_plugin` emits the same
  shape from pytest.

Colours, glyphs, suite headers (10 × U+2500 each side) and the summary line
(40 × ``=``; `` PASS  All N checks passed`` / `` FAIL  k failed, n passed``) are the
reference's.  Difference: the reference decides the mode from line 0 only, so ``go test -json``
(whose first event is a package-level ``start`` without ``Test``) never enters test mode
(SURVEY.md §2.5 #14); here the first *parseable* line decides and ``Action`` also counts.
Test-mode durations come from the event's ``Elapsed`` when present, else the local clock.
"""
from __future__ import annotations

import json
import sys
import time
from typing import IO, Dict, Iterable, List, Optional

GREEN = "\033[0;32m"
RED = "\033[0;31m"
GRAY = "\033[0;90m"
CYAN = "\033[0;36m"
BOLD = "\033[1m"
RESET = "\033[0m"
BG_GREEN = "\033[42;30m"
BG_RED = "\033[41;37m"


class _State:
    def __init__(self, out: IO[str]):
        self.out = out
        self.current_suite = ""
        self.failures: List[str] = []
        self.passes = 0
        self.tests: Dict[str, float] = {}

    def w(self, s: str) -> None:
        self.out.write(s)


def suite_header(st: _State, name: str) -> None:
    if st.current_suite != name:
        sep = "─" * 10
        st.w(f"\n{GRAY}{sep} {BOLD}{name} {sep}{RESET}\n")
        st.current_suite = name


def step(st: _State, status: str, message: str, details: str = "") -> None:
    color, symbol = (GREEN, "✓") if status == "PASS" else (RED, "✗")
    if details:
        st.w(f"  {color}{symbol}{RESET} {message} {GRAY}({details}){RESET}\n")
    else:
        st.w(f"  {color}{symbol}{RESET} {message}\n")


def _v(x) -> str:
    """Go's ``%v`` of a JSON-decoded value."""
    if x is None:
        return "<nil>"
    if isinstance(x, bool):
        return "true" if x else "false"
    if isinstance(x, float) and x.is_integer():
        return str(int(x))
    if isinstance(x, dict):
        return "map[" + " ".join(f"{k}:{_v(v)}" for k, v in sorted(x.items())) + "]"
    if isinstance(x, list):
        return "[" + " ".join(_v(v) for v in x) + "]"
    return str(x)


def _app_entry(e: dict, st: _State) -> None:
    msg = e.get("msg", "") if isinstance(e.get("msg"), str) else ""
    level = e.get("level", "") if isinstance(e.get("level"), str) else ""
    if level == "DEBUG":
        suite_header(st, "CONNECTION")
        st.w(f"    {GRAY}{msg} ...state={_v(e.get('state'))}{RESET}\n")
        return
    if msg == "Configuration loaded":
        suite_header(st, "SETUP")
        step(st, "PASS", "Configuration", f"server={_v(e.get('server'))}")
        st.passes += 1
    elif msg == "Network connectivity test passed":
        suite_header(st, "CONNECTION")
        step(st, "PASS", "Network Connectivity")
        st.passes += 1
    elif msg == "gRPC connection established successfully":
        suite_header(st, "CONNECTION")
        step(st, "PASS", "gRPC Connection")
        st.passes += 1
    elif msg == "Executing tool":
        suite_header(st, "EXECUTION")
        step(st, "PASS", "Tool Execution", f"tool={_v(e.get('tool_name'))}")
        st.passes += 1
    elif msg == "Tool execution completed":
        suite_header(st, "EXECUTION")
        st.w(f"    {GRAY}└─ Status: {CYAN}'{_v(e.get('status_message'))}'{RESET}\n")
    elif msg == "Received struct output":
        suite_header(st, "EXECUTION")
        st.w(f"    {GRAY}└─ Received Output {GRAY}(fields={_v(e.get('field_count'))}){RESET}\n")
    elif msg == "Application failed":
        suite_header(st, "ERROR")
        details = _v(e.get("error"))
        step(st, "FAIL", "Application Run", details)
        st.failures.append(f"Application failed: {details}")


def _go_duration_ms(seconds: float) -> str:
    from ..utils.slog import go_duration
    return go_duration(round(seconds, 3))


def _test_entry(e: dict, st: _State) -> None:
    action = e.get("Action", "") or ""
    test = e.get("Test", "") or ""
    pkg = e.get("Package", "") or ""
    if not test:
        return
    if action == "run":
        suite_header(st, pkg)
        st.tests[test] = time.monotonic()
        st.w(f"  ○ {GRAY}{test}\n")
    elif action in ("pass", "fail"):
        if isinstance(e.get("Elapsed"), (int, float)):
            dur = float(e["Elapsed"])
        else:
            dur = time.monotonic() - st.tests.get(test, time.monotonic())
        step(st, "PASS" if action == "pass" else "FAIL", test, _go_duration_ms(dur))
        if action == "pass":
            st.passes += 1
        else:
            st.failures.append(test)


def summary(st: _State) -> None:
    st.w(GRAY + "\n" + "=" * 40 + RESET + "\n")
    if st.failures:
        st.w(f" {BG_RED} FAIL {RESET} {len(st.failures)} failed, {st.passes} passed\n")
    else:
        st.w(f" {BG_GREEN} PASS {RESET} All {st.passes} checks passed\n")


def print_jest_report(lines: Iterable[str], out: Optional[IO[str]] = None,
                      title_app: str = "Polykey Dev Client", title_test: str = "Go Test Suite") -> int:
    """Render ``lines``; returns the number of failures."""
    st = _State(out or sys.stdout)
    st.w("\n")
    mode: Optional[str] = None
    for line in lines:
        if not line:
            continue
        try:
            e = json.loads(line)
        except ValueError:
            continue
        if not isinstance(e, dict):
            continue
        if mode is None:
            if "Test" in e or "Action" in e:
                mode = "test"
                st.w(f"{BOLD}{CYAN} RUNS {title_test}{RESET}\n")
            elif "msg" in e:
                mode = "app"
                st.w(f"{BOLD}{CYAN} RUNS {title_app}{RESET}\n")
            else:
                continue
        if mode == "test":
            _test_entry(e, st)
        else:
            _app_entry(e, st)
    summary(st)
    return len(st.failures)


def main(argv=None) -> int:
    """``python -m polykey_service_amd.report.jest < logs.jsonl``"""
    return 1 if print_jest_report(sys.stdin.read().split("\n")) else 0


if __name__ == "__main__":
    raise SystemExit(main())
