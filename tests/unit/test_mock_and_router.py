"""MockService golden outputs (reference internal/service/mock.go:22-67) + ToolRouter."""
import asyncio
import datetime as dt
import re
import time

import pytest

from polykey_service_amd import proto
from polykey_service_amd.service import MockService, RequestContext, ToolError, ToolRouter, rfc3339_now


def run(coro):
    return asyncio.run(coro)


def call(svc, name, **kw):
    return run(svc.execute_tool(RequestContext(), name, kw.get("params"), kw.get("secret"), kw.get("md")))


@pytest.mark.parametrize("svc_factory", [MockService, ToolRouter])
def test_status_always_200(svc_factory):
    for name in ("example_tool", "struct_tool", "file_tool", "nope"):
        r = call(svc_factory(), name)
        assert r.status.code == 200 and r.status.message == "Tool executed successfully"


@pytest.mark.parametrize("svc_factory", [MockService, ToolRouter])
def test_example_tool(svc_factory):
    r = call(svc_factory(), "example_tool")
    assert r.WhichOneof("output") == "string_output"
    m = re.fullmatch(r"Mock execution of example_tool at (\S+)", r.string_output)
    assert m and re.fullmatch(r"\d{4}-\d\d-\d\dT\d\d:\d\d:\d\d(Z|[+-]\d\d:\d\d)", m.group(1))


@pytest.mark.parametrize("svc_factory", [MockService, ToolRouter])
def test_struct_tool(svc_factory):
    t0 = int(time.time())
    r = call(svc_factory(), "struct_tool")
    d = proto.struct_to_dict(r.struct_output)
    assert d["result"] == "success" and d["data"] == {"processed": True, "count": 42.0}
    assert t0 <= d["timestamp"] <= t0 + 2 and set(d) == {"result", "timestamp", "data"}


@pytest.mark.parametrize("svc_factory", [MockService, ToolRouter])
def test_file_tool(svc_factory):
    f = call(svc_factory(), "file_tool").file_output
    assert (f.file_name, f.mime_type, f.content) == ("example.txt", "text/plain", b"This is mock file content")


@pytest.mark.parametrize("svc_factory", [MockService, ToolRouter])
def test_unknown_tool(svc_factory):
    assert call(svc_factory(), "weird name").string_output == "Unknown tool: weird name"
    assert call(svc_factory(), "").string_output == "Unknown tool: "


def test_params_secret_metadata_ignored_by_mock():
    md = proto.Metadata()
    md.fields["a"] = "b"
    r = call(MockService(), "file_tool", params=proto.struct_from_dict({"x": 1}), secret="s", md=md)
    assert r.file_output.file_name == "example.txt"


def test_rfc3339_formats():
    utc = dt.datetime(2025, 7, 18, 1, 2, 3, tzinfo=dt.timezone.utc)
    assert rfc3339_now(utc) == "2025-07-18T01:02:03Z"
    tz = dt.timezone(dt.timedelta(hours=-5, minutes=-30))
    assert rfc3339_now(utc.astimezone(tz)) == "2025-07-17T19:32:03-05:30"


class EchoTool:
    requires_secret = False

    def __init__(self, name):
        self.name = name

    async def run(self, ctx, params, secret, md):
        r = proto.ExecuteToolResponse(status=proto.Status(code=200, message="ok"))
        r.string_output = f"{self.name}:{params.get('prompt', '')}:{md.get('k', '')}"
        return r

    async def stream(self, ctx, params, secret, md):
        for i in range(3):
            yield proto.ExecuteToolResponse(string_output=str(i))


class SecretTool(EchoTool):
    requires_secret = True

    async def run(self, ctx, params, secret, md):
        return proto.ExecuteToolResponse(string_output=secret.decode())


def test_router_model_family_routing():
    r = ToolRouter()
    r.register_model_tool("llm.chat", "llama3-8b", EchoTool("llama"))
    r.register_model_tool("llm.chat", "mixtral-8x7b", EchoTool("mixtral"))
    assert call(r, "llm.chat", params=proto.struct_from_dict({"prompt": "p"})).string_output == "llama:p:"
    assert call(r, "llm.chat:mixtral-8x7b").string_output == "mixtral::"
    assert call(r, "llm.chat", params=proto.struct_from_dict({"model": "mixtral-8x7b"})).string_output == "mixtral::"
    with pytest.raises(ToolError) as ei:
        call(r, "llm.chat:gpt-9")
    assert ei.value.code == "NOT_FOUND"
    assert "llm.chat:mixtral-8x7b" in r.tools()


def test_router_stream():
    r = ToolRouter()
    r.register(EchoTool("echo"))

    async def collect():
        return [c.string_output async for c in r.execute_tool_stream(RequestContext(), "echo")]

    assert run(collect()) == ["0", "1", "2"]


def test_router_secret_resolution():
    from polykey_service_amd.adapters.security import SecretStore
    store = SecretStore(b"m" * 32)
    store.put("sk-1", b"provider-key")
    r = ToolRouter(secret_store=store)
    r.register(SecretTool("paid"))
    assert call(r, "paid", secret="sk-1").string_output == "provider-key"
    with pytest.raises(ToolError) as ei:
        call(r, "paid")
    assert ei.value.code == "UNAUTHENTICATED"
    with pytest.raises(ToolError) as ei:
        call(r, "paid", secret="missing")
    assert ei.value.code == "NOT_FOUND"
