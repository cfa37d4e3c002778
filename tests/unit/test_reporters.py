"""Golden-output tests for the Jest reporter (beautify.go) and server log filter (log-beautifier)."""
import io
import json

from polykey_service_amd.report.jest import print_jest_report
from polykey_service_amd.report.log_beautifier import ERASE_LINE, Beautifier

G, R, GR, C, B, X = "\033[0;32m", "\033[0;31m", "\033[0;90m", "\033[0;36m", "\033[1m", "\033[0m"


def J(**kw):
    return json.dumps(kw)


def header(name):
    return f"\n{GR}{'─' * 10} {B}{name} {'─' * 10}{X}\n"


def test_app_mode_golden():
    lines = [
        J(time="t", level="INFO", msg="Starting polykey client..."),
        J(time="t", level="INFO", msg="Configuration loaded", runtime="local", server="localhost:50051"),
        J(time="t", level="INFO", msg="Network connectivity test passed"),
        J(time="t", level="DEBUG", msg="Initial connection state", state="IDLE"),
        J(time="t", level="INFO", msg="gRPC connection established successfully"),
        J(time="t", level="INFO", msg="Executing tool", tool_name="example_tool"),
        J(time="t", level="INFO", msg="Tool execution completed", status_code=200, status_message="Tool executed successfully"),
        J(time="t", level="INFO", msg="Received struct output", field_count=3),
        "", "not json",
    ]
    out = io.StringIO()
    assert print_jest_report(lines, out) == 0
    exp = ("\n" + f"{B}{C} RUNS Polykey Dev Client{X}\n"
           + header("SETUP") + f"  {G}✓{X} Configuration {GR}(server=localhost:50051){X}\n"
           + header("CONNECTION") + f"  {G}✓{X} Network Connectivity\n"
           + f"    {GR}Initial connection state ...state=IDLE{X}\n"
           + f"  {G}✓{X} gRPC Connection\n"
           + header("EXECUTION") + f"  {G}✓{X} Tool Execution {GR}(tool=example_tool){X}\n"
           + f"    {GR}└─ Status: {C}'Tool executed successfully'{X}\n"
           + f"    {GR}└─ Received Output {GR}(fields=3){X}\n"
           + f"{GR}\n{'=' * 40}{X}\n" + f" \033[42;30m PASS {X} All 4 checks passed\n")
    assert out.getvalue() == exp


def test_app_mode_failure():
    out = io.StringIO()
    n = print_jest_report([J(level="INFO", msg="Configuration loaded", server="s"),
                           J(level="ERROR", msg="Application failed", error="boom")], out)
    assert n == 1
    s = out.getvalue()
    assert header("ERROR") in s and f"  {R}✗{X} Application Run {GR}(boom){X}\n" in s
    assert s.endswith(f" \033[41;37m FAIL {X} 1 failed, 1 passed\n")


def test_test_mode_go_test_json_with_package_start_first():
    lines = [J(Action="start", Package="p"),  # go test -json starts without Test
             J(Action="run", Package="p", Test="TestA"), J(Action="pass", Package="p", Test="TestA", Elapsed=0.25),
             J(Action="run", Package="p", Test="TestB"), J(Action="fail", Package="p", Test="TestB", Elapsed=1.5)]
    out = io.StringIO()
    assert print_jest_report(lines, out) == 1
    s = out.getvalue()
    assert "RUNS Go Test Suite" in s and header("p") in s
    assert f"  {G}✓{X} TestA {GR}(250ms){X}\n" in s and f"  {R}✗{X} TestB {GR}(1.5s){X}\n" in s
    assert "1 failed, 1 passed" in s


def test_beautifier_golden_and_concurrency():
    out = io.StringIO()
    t = iter([0.0, 0.010, 0.020, 0.5]).__next__
    b = Beautifier(out, clock=t)
    b.run([
        'polykey-server-1  | ' + J(msg="server starting", address=":50051"),
        "plain text line",
        J(msg="gRPC call received", method="/m", request_id=1),
        J(msg="gRPC call received", method="/m", request_id=2),
        J(msg="gRPC call finished", method="/m", code="OK", request_id=1, duration="x"),
        J(msg="gRPC call finished", method="/m", code="Unknown", request_id=2, duration="x"),
        J(msg="gRPC call finished", method="/never", code="OK"),
        J(msg="server shutting down"), J(msg="server stopped"),
    ])
    s = out.getvalue()
    assert header("SETUP") in s and f"{ERASE_LINE}  {G}✓{X} Server Listening {GR}(addr=:50051){X}\n" in s
    assert "plain text line\n" in s
    assert f"{ERASE_LINE}  {G}✓{X} /m {GR}(20ms){X}\n" in s  # keyed by request_id, not method
    assert f"{ERASE_LINE}  {R}✗{X} /m {GR}(490ms){X}\n" in s
    assert "/never" not in s
    assert header("SHUTDOWN") in s and s.endswith(f"{ERASE_LINE}  {G}✓{X} server stopped\n")
