"""Integration tests against a running server at ``POLYKEY_SERVER_ADDR`` (the container flow
of ``make test-integration`` / the CI ``integration-test`` job, mirroring the reference's
``go test -tags=integration`` run against the compose service); skipped when unset.  The
health-probe CLI is also checked in-process here."""
import os
import subprocess
import sys

import grpc
import pytest

from polykey_service_amd import proto
from polykey_service_amd.client.health_probe import probe
from polykey_service_amd.service.mock import MockService
from tests.helpers import ServerThread

ADDR = os.environ.get("POLYKEY_SERVER_ADDR")
remote = pytest.mark.skipif(not ADDR, reason="POLYKEY_SERVER_ADDR not set (no server container)")


def test_health_probe_cli_against_in_process_server():
    with ServerThread(MockService()) as s:
        assert probe(s.addr) == 0
        assert probe(s.addr, service="no.such.Service") == 3
        r = subprocess.run([sys.executable, "-m", "polykey_service_amd.client.health_probe", f"-addr={s.addr}",
                            "-connect-timeout=5s"], capture_output=True, text=True, timeout=60)
        assert r.returncode == 0 and "SERVING" in r.stdout
    assert probe("127.0.0.1:1", timeout_s=0.5) == 2


@remote
def test_remote_health_and_example_tool():
    assert probe(ADDR) == 0
    with grpc.insecure_channel(ADDR) as ch:
        call = ch.unary_unary(proto.EXECUTE_TOOL, request_serializer=proto.ExecuteToolRequest.SerializeToString,
                              response_deserializer=proto.ExecuteToolResponse.FromString)
        r = call(proto.ExecuteToolRequest(tool_name="example_tool"), timeout=30)
        assert r.status.code == 200 and r.string_output.startswith("Mock execution of example_tool at ")
        r = call(proto.ExecuteToolRequest(tool_name="struct_tool"), timeout=30)
        assert proto.struct_to_dict(r.struct_output)["result"] == "success"
        r = call(proto.ExecuteToolRequest(tool_name="nope"), timeout=30)
        assert r.string_output == "Unknown tool: nope"
