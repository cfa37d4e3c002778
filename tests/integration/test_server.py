"""In-process grpc.aio server on an ephemeral port (config 1: dev_client example_tool vs mock, CPU)."""
import asyncio
import io
import json
import threading
import time

import grpc
import pytest

from polykey_service_amd import proto
from polykey_service_amd.client import dev_client
from polykey_service_amd.proto import schema
from polykey_service_amd.server import NOT_SERVING, SERVING, PolykeyServer
from polykey_service_amd.service import ToolError, ToolRouter
from polykey_service_amd.utils import slog
from tests.helpers import ServerThread


def unary(ch, method, req_cls, resp_cls):
    return ch.unary_unary(method, request_serializer=req_cls.SerializeToString,
                          response_deserializer=resp_cls.FromString)


def test_execute_tool_and_interceptor_schema():
    with ServerThread() as s, grpc.insecure_channel(s.addr) as ch:
        call = unary(ch, proto.EXECUTE_TOOL, proto.ExecuteToolRequest, proto.ExecuteToolResponse)
        r = call(dev_client.build_request("struct_tool"), timeout=5)
        assert r.status.code == 200 and r.WhichOneof("output") == "struct_output"
        hc = unary(ch, proto.HEALTH_CHECK, proto.HealthCheckRequest, proto.HealthCheckResponse)
        assert hc(proto.HealthCheckRequest(service=""), timeout=5).status == SERVING
        recs = s.records()
    msgs = [r["msg"] for r in recs]
    assert msgs[0] == "Registered services:" and "server starting" in msgs
    methods = {(r["service"], r["method"]) for r in recs if r["msg"] == "Method available"}
    assert ("polykey.v2.PolykeyService", "ExecuteTool") in methods
    got = [r for r in recs if r["msg"].startswith("gRPC call")]
    # Health/Check bypasses the interceptor (main.go:29-31)
    assert [r["msg"] for r in got] == ["gRPC call received", "gRPC call finished"]
    fin = got[1]
    assert fin["method"] == "/polykey.v2.PolykeyService/ExecuteTool" and fin["code"] == "OK"
    assert fin["level"] == "INFO" and fin["duration"].endswith("s")
    called = [r for r in recs if r["msg"] == "ExecuteTool called"][0]
    assert called == {**called, "tool_name": "struct_tool", "has_parameters": True, "has_secret_id": True,
                      "has_metadata": True}


class FailingService(ToolRouter):
    async def execute_tool(self, ctx, tool_name, parameters=None, secret_id=None, metadata=None):
        if tool_name == "raise":
            raise RuntimeError("kaput")
        raise ToolError("INVALID_ARGUMENT", "bad params")


def test_errors_map_to_codes_and_error_logs():
    with ServerThread(FailingService()) as s, grpc.insecure_channel(s.addr) as ch:
        call = unary(ch, proto.EXECUTE_TOOL, proto.ExecuteToolRequest, proto.ExecuteToolResponse)
        with pytest.raises(grpc.RpcError) as ei:
            call(proto.ExecuteToolRequest(tool_name="raise"), timeout=5)
        assert ei.value.code() == grpc.StatusCode.UNKNOWN and "kaput" in ei.value.details()
        with pytest.raises(grpc.RpcError) as ei:
            call(proto.ExecuteToolRequest(tool_name="x"), timeout=5)
        assert ei.value.code() == grpc.StatusCode.INVALID_ARGUMENT
        recs = s.records()
    fins = [r for r in recs if r["msg"] == "gRPC call finished"]
    assert [(r["level"], r["code"]) for r in fins] == [("ERROR", "Unknown"), ("ERROR", "InvalidArgument")]
    assert any(r["msg"] == "Service ExecuteTool failed" and r["error"] == "kaput" for r in recs)


def test_unimplemented_method():
    with ServerThread() as s, grpc.insecure_channel(s.addr) as ch:
        call = unary(ch, "/polykey.v2.PolykeyService/Nope", proto.ExecuteToolRequest, proto.ExecuteToolResponse)
        with pytest.raises(grpc.RpcError) as ei:
            call(proto.ExecuteToolRequest(), timeout=5)
        assert ei.value.code() == grpc.StatusCode.UNIMPLEMENTED


def test_streaming_rpc_mock():
    with ServerThread() as s, grpc.insecure_channel(s.addr) as ch:
        st = ch.unary_stream(proto.EXECUTE_TOOL_STREAM, request_serializer=proto.ExecuteToolRequest.SerializeToString,
                             response_deserializer=proto.ExecuteToolResponse.FromString)
        out = list(st(proto.ExecuteToolRequest(tool_name="file_tool"), timeout=5))
        assert len(out) == 1 and out[0].file_output.content == b"This is mock file content"


def test_health_unknown_watch_and_shutdown():
    with ServerThread() as s, grpc.insecure_channel(s.addr) as ch:
        hc = unary(ch, proto.HEALTH_CHECK, proto.HealthCheckRequest, proto.HealthCheckResponse)
        assert hc(proto.HealthCheckRequest(service="polykey.v2.PolykeyService"), timeout=5).status == SERVING
        with pytest.raises(grpc.RpcError) as ei:
            hc(proto.HealthCheckRequest(service="nope"), timeout=5)
        assert ei.value.code() == grpc.StatusCode.NOT_FOUND
        watch = ch.unary_stream(proto.HEALTH_WATCH, request_serializer=proto.HealthCheckRequest.SerializeToString,
                                response_deserializer=proto.HealthCheckResponse.FromString)
        it = watch(proto.HealthCheckRequest(service=""), timeout=10)
        assert next(it).status == SERVING
        s.loop.call_soon_threadsafe(s.srv.health.shutdown)
        assert next(it).status == NOT_SERVING
        it.cancel()
        s.stop(0.5)
        msgs = [r["msg"] for r in s.records()]
    assert msgs[-1] == "server stopped" and "server shutting down" in msgs


def test_reflection_list_and_describe():
    from google.protobuf import descriptor_pb2
    Req = schema.message_class("grpc.reflection.v1alpha.ServerReflectionRequest")
    Resp = schema.message_class("grpc.reflection.v1alpha.ServerReflectionResponse")
    with ServerThread() as s, grpc.insecure_channel(s.addr) as ch:
        rpc = ch.stream_stream("/grpc.reflection.v1alpha.ServerReflection/ServerReflectionInfo",
                               request_serializer=Req.SerializeToString, response_deserializer=Resp.FromString)
        reqs = [Req(list_services=""), Req(file_containing_symbol="polykey.v2.PolykeyService"),
                Req(file_by_filename="common/v2/common.proto"), Req(file_containing_symbol="no.Such")]
        out = list(rpc(iter(reqs), timeout=5))
    names = [x.name for x in out[0].list_services_response.service]
    assert "polykey.v2.PolykeyService" in names and "grpc.health.v1.Health" in names
    files = [descriptor_pb2.FileDescriptorProto.FromString(b) for b in
             out[1].file_descriptor_response.file_descriptor_proto]
    fnames = [f.name for f in files]
    assert fnames[0] == "polykey/v2/polykey.proto" and "google/protobuf/struct.proto" in fnames
    assert "common/v2/common.proto" in fnames
    svc = files[0].service[0]
    assert [m.name for m in svc.method] == ["ExecuteTool", "ExecuteToolStream"]
    assert out[2].file_descriptor_response.file_descriptor_proto
    assert out[3].WhichOneof("message_response") == "error_response"


def test_dev_client_end_to_end(monkeypatch):
    with ServerThread() as s:
        monkeypatch.setenv("POLYKEY_SERVER_ADDR", s.addr)
        out = io.StringIO()
        assert dev_client.main([], out=out) == 0
        text = out.getvalue()
    assert "All 4 checks passed" in text and "tool=example_tool" in text
    assert "'Tool executed successfully'" in text


def test_dev_client_fails_without_server(monkeypatch):
    monkeypatch.setenv("POLYKEY_SERVER_ADDR", "127.0.0.1:1")
    out = io.StringIO()
    assert dev_client.main([], out=out) == 1
    assert "Application Run" in out.getvalue() and "network test failed" in out.getvalue()


def test_keepalive_enforcement_allows_10s_pings():
    from polykey_service_amd.server import SERVER_OPTIONS
    opts = dict(SERVER_OPTIONS)
    assert opts["grpc.http2.min_recv_ping_interval_without_data_ms"] <= 10_000
    assert opts["grpc.keepalive_permit_without_calls"] == 1
    assert opts["grpc.max_connection_idle_ms"] == 300_000 and opts["grpc.keepalive_time_ms"] == 7_200_000


class SlowStreamService(ToolRouter):
    """A stream of 5 chunks, 0.1 s apart (an LLM stream in flight when the server stops)."""

    def __init__(self):
        super().__init__()
        self.started = threading.Event()

    async def execute_tool_stream(self, ctx, tool_name, parameters=None, secret_id=None, metadata=None):
        for i in range(5):
            self.started.set()
            yield proto.ExecuteToolResponse(string_output=f"chunk{i}")
            await asyncio.sleep(0.1)


def test_graceful_shutdown_lets_in_flight_streams_finish():
    """SIGTERM path (R7): health flips to NOT_SERVING first, new calls are refused, and a stream
    already in flight still delivers every chunk within the grace period."""
    svc = SlowStreamService()
    with ServerThread(svc) as s, grpc.insecure_channel(s.addr) as ch:
        st = ch.unary_stream(proto.EXECUTE_TOOL_STREAM, request_serializer=proto.ExecuteToolRequest.SerializeToString,
                             response_deserializer=proto.ExecuteToolResponse.FromString)
        got = []
        reader = threading.Thread(target=lambda: got.extend(
            r.string_output for r in st(proto.ExecuteToolRequest(tool_name="slow"), timeout=10)))
        reader.start()
        assert svc.started.wait(5)
        stopper = threading.Thread(target=s.stop, args=(5.0,))
        stopper.start()
        reader.join(10)
        stopper.join(10)
        assert got == [f"chunk{i}" for i in range(5)]
        assert s.srv.health.get("") == NOT_SERVING
        with pytest.raises(grpc.RpcError):
            unary(ch, proto.EXECUTE_TOOL, proto.ExecuteToolRequest, proto.ExecuteToolResponse)(
                proto.ExecuteToolRequest(tool_name="example_tool"), timeout=2)
        msgs = [r["msg"] for r in s.records()]
    assert msgs.index("server shutting down") < msgs.index("server stopped")


def test_keepalive_10s_pings_on_a_live_connection_get_no_goaway():
    """SURVEY §2.5 #10 / §4.2, live: a dev_client-style channel pinging every 10 s
    (keepalive_time 10 s, permit without calls: /root/reference/cmd/dev_client/main.go:182-186)
    stays on ONE connection for > 30 s against our server.  Control: the same client against a
    server with grpc's default enforcement (no ping-interval setting, 2 ping strikes) is sent
    GOAWAY too_many_pings in that time -- so the check can see the failure it guards against."""
    import grpc

    from polykey_service_amd.server import app

    client_opts = [("grpc.keepalive_time_ms", 10_000), ("grpc.keepalive_timeout_ms", 5_000),
                   ("grpc.keepalive_permit_without_calls", 1), ("grpc.http2.max_pings_without_data", 0)]
    default_enforcement = [o for o in app.SERVER_OPTIONS if o[0] not in (
        "grpc.http2.min_recv_ping_interval_without_data_ms", "grpc.http2.max_ping_strikes")]

    def watch(addr):
        ch = grpc.insecure_channel(addr, options=client_opts)
        states = []
        ch.subscribe(lambda s: states.append(s), try_to_connect=True)
        grpc.channel_ready_future(ch).result(timeout=10)
        call = ch.unary_unary(proto.EXECUTE_TOOL, request_serializer=proto.ExecuteToolRequest.SerializeToString,
                              response_deserializer=proto.ExecuteToolResponse.FromString)
        assert call(proto.ExecuteToolRequest(tool_name="example_tool"), timeout=10).status.code == 200
        return ch, states, call

    saved = app.SERVER_OPTIONS
    with ServerThread() as ours:
        try:
            app.SERVER_OPTIONS = default_enforcement
            control = ServerThread().__enter__()
        finally:
            app.SERVER_OPTIONS = saved
        chans = []
        try:
            ch1, st1, call1 = watch(ours.addr)
            ch2, st2, _ = watch(control.addr)
            chans += [ch1, ch2]
            time.sleep(36)  # three or more 10 s pings with no data in between
            after_ready = lambda st: st[st.index(grpc.ChannelConnectivity.READY) + 1:]
            assert after_ready(st1) == [], st1  # never left READY: no GOAWAY, no reconnect
            assert call1(proto.ExecuteToolRequest(tool_name="example_tool"), timeout=10).status.code == 200
            assert any(s != grpc.ChannelConnectivity.READY for s in after_ready(st2)), st2  # control was cut
        finally:
            for ch in chans:
                ch.close()
            control.__exit__(None, None, None)
