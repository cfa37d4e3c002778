"""Tool calling on the chat route (BASELINE.json config 5 "tool-call routing path"): chat
templates, call parsing, forced calls with the real tiny models, and parsed calls routed to the
gateway's own tools (mock and secret-gated) over OpenAI HTTP and gRPC."""
import json
import os

import grpc
import pytest

from polykey_service_amd import proto
from polykey_service_amd.adapters.local_llm import LLMTool, attach_local_llm
from polykey_service_amd.adapters.security.secret_store import SecretStore
from polykey_service_amd.config.server_config import ServerConfig
from polykey_service_amd.engine import EngineConfig, LLMEngine
from polykey_service_amd.engine.chat_template import LLAMA3, MISTRAL, ChatTemplate, load_chat_template
from polykey_service_amd.engine.sequence import RequestOutput
from polykey_service_amd.engine.tokenizer import ByteTokenizer
from polykey_service_amd.parallel.state import ParallelState
from polykey_service_amd.service import ToolRouter
from polykey_service_amd.service.tool_calls import forced_call, parse_tool_calls
from polykey_service_amd.utils import slog

from tests.helpers import ServerThread

WEATHER = {"type": "function", "function": {"name": "get_weather", "description": "current weather",
                                            "parameters": {"type": "object",
                                                           "properties": {"city": {"type": "string"}}}}}
EXAMPLE = {"type": "function", "function": {"name": "example_tool", "parameters": {"type": "object"}}}
VAULT = {"type": "function", "function": {"name": "vault_tool", "parameters": {"type": "object"}}}


# ------------------------------------------------------------------ templates / parsing
def test_llama3_template_with_tools_and_results():
    t = ChatTemplate(LLAMA3)
    msgs = [{"role": "system", "content": "be brief"}, {"role": "user", "content": "weather in Oslo?"},
            {"role": "assistant", "content": None,
             "tool_calls": [{"id": "c1", "type": "function",
                             "function": {"name": "get_weather", "arguments": "{\"city\": \"Oslo\"}"}}]},
            {"role": "tool", "tool_call_id": "c1", "content": "sunny"}]
    s = t.render(msgs, [WEATHER])
    assert s.startswith("<|start_header_id|>system<|end_header_id|>\n\nEnvironment: ipython\nbe brief")
    assert '"name": "get_weather"' in s and "<|python_tag|>{\"name\": \"get_weather\", \"parameters\": " \
                                           "{\"city\": \"Oslo\"}}<|eom_id|>" in s
    assert "<|start_header_id|>ipython<|end_header_id|>\n\nsunny<|eot_id|>" in s
    assert s.endswith("<|start_header_id|>assistant<|end_header_id|>\n\n")
    assert t.render([{"role": "user", "content": "hi"}]) == \
        "<|start_header_id|>user<|end_header_id|>\n\nhi<|eot_id|><|start_header_id|>assistant<|end_header_id|>\n\n"


def test_mistral_template_with_tools_and_results():
    t = ChatTemplate(MISTRAL)
    msgs = [{"role": "user", "content": "a"}, {"role": "assistant", "content": "b"},
            {"role": "user", "content": "weather?"},
            {"role": "assistant", "tool_calls": [{"id": "c9", "function": {"name": "get_weather",
                                                                           "arguments": {"city": "Rome"}}}]},
            {"role": "tool", "tool_call_id": "c9", "content": "rain"}]
    s = t.render(msgs, [WEATHER])
    assert s.startswith("[INST] a [/INST]b</s>[AVAILABLE_TOOLS] [")
    assert "[/AVAILABLE_TOOLS][INST] weather? [/INST][TOOL_CALLS] [{\"name\": \"get_weather\", \"arguments\": " \
           "{\"city\": \"Rome\"}}]</s>[TOOL_RESULTS] {\"content\": \"rain\", \"call_id\": \"c9\"}[/TOOL_RESULTS]" in s


def test_hf_jinja_template_from_tokenizer_dir(tmp_path):
    src = ("{% for m in messages %}<{{ m['role'] }}>{{ m['content'] }}{% endfor %}"
           "{% if tools %}[TOOLS]{{ tools | tojson }}{% endif %}{% if add_generation_prompt %}<assistant>{% endif %}")
    (tmp_path / "tokenizer_config.json").write_text(json.dumps({"chat_template": src, "eos_token": "</s>"}))
    t = load_chat_template(str(tmp_path), LLAMA3)
    assert t.jinja_source == src
    out = t.render([{"role": "user", "content": "q"}], [WEATHER])
    assert out.startswith("<user>q[TOOLS]") and out.endswith("<assistant>")
    # no template in the directory: the family's built-in one
    assert load_chat_template(str(tmp_path / "missing"), MISTRAL).family == MISTRAL


def test_parse_tool_call_formats():
    names = ["get_weather", "example_tool"]
    c, calls = parse_tool_calls('{"name": "get_weather", "parameters": {"city": "Oslo"}}<|eom_id|>', names)
    assert c == "" and calls[0]["function"] == {"name": "get_weather", "arguments": '{"city": "Oslo"}'}
    assert calls[0]["type"] == "function" and calls[0]["id"].startswith("call_")
    _, calls = parse_tool_calls('<|python_tag|>{"name": "example_tool", "parameters": {}}; '
                                '{"name": "get_weather", "arguments": {"city": "Rome"}}', names)
    assert [x["function"]["name"] for x in calls] == ["example_tool", "get_weather"]
    c, calls = parse_tool_calls('Let me check. [TOOL_CALLS] [{"name": "get_weather", "arguments": {"city": "X"}}]</s>',
                                names)
    assert c == "Let me check." and json.loads(calls[0]["function"]["arguments"]) == {"city": "X"}
    _, calls = parse_tool_calls('<tool_call>{"name": "example_tool", "arguments": {"a": 1}}</tool_call>', names)
    assert calls[0]["function"]["name"] == "example_tool"
    # unknown functions, prose and broken JSON stay content
    assert parse_tool_calls('{"name": "rm_rf", "parameters": {}}', names)[1] == []
    assert parse_tool_calls("it is sunny", names) == ("it is sunny", [])
    assert parse_tool_calls('{"name": "get_weather", "parameters": {"city": ', names)[1] == []
    assert parse_tool_calls('{"name": "get_weather", "parameters": {}} and more', names)[1] == []


def test_forced_call_arguments():
    c = forced_call('{"city": "Oslo"}}<|eom_id|>', "get_weather", ["get_weather"], LLAMA3)
    assert c["function"] == {"name": "get_weather", "arguments": '{"city": "Oslo"}'}
    # not valid JSON: the model's own text is the arguments string (OpenAI semantics)
    assert forced_call("xyz}", "get_weather", ["get_weather"], LLAMA3)["function"]["arguments"] == "xyz"
    # the model picked the name
    c = forced_call('example_tool", "arguments": {"q": 1}}]', None, ["get_weather", "example_tool"], MISTRAL)
    assert c["function"] == {"name": "example_tool", "arguments": '{"q": 1}'}


# ------------------------------------------------------------------ scripted model, routed calls
class _ScriptedLLM:
    """Duck-types AsyncLLM: replies with scripted texts in turn and records the prompts."""

    def __init__(self, replies, family=LLAMA3):
        self.tokenizer = ByteTokenizer(1024, chat_template=ChatTemplate(family))
        self.replies = list(replies)
        self.prompts = []

    async def generate_all(self, prompt_ids, params, request_id=None):
        self.prompts.append(self.tokenizer.decode(prompt_ids))
        toks = self.tokenizer.encode(self.replies.pop(0), add_bos=False)
        return toks, RequestOutput(request_id or "r", toks[-1:], True, "stop", len(prompt_ids), len(toks), {})

    def healthy(self):
        return True


class _VaultTool:
    name = "vault_tool"
    requires_secret = True

    async def run(self, ctx, params, secret, metadata):
        return proto.ExecuteToolResponse(status=proto.Status(code=200, message="ok"),
                                         string_output=f"vault opened with {len(secret)}-byte key")

    async def stream(self, ctx, params, secret, metadata):
        yield await self.run(ctx, params, secret, metadata)


def _scripted_router(replies, family=LLAMA3):
    store = SecretStore(os.urandom(32))
    store.put("sid-1", b"0123456789")
    r = ToolRouter(secret_store=store)
    r.register(_VaultTool())
    llm = _ScriptedLLM(replies, family)
    r.register_model_tool("llm.chat", "scripted", tool := LLMTool("llm.chat", "scripted", llm, chat=True))
    tool.router = r
    return r, llm


def test_openai_parsed_call_returned_to_client():
    from fastapi.testclient import TestClient

    from polykey_service_amd.api.openai import create_app
    router, llm = _scripted_router(['{"name": "get_weather", "parameters": {"city": "Oslo"}}'])
    c = TestClient(create_app(router))
    r = c.post("/v1/chat/completions", json={"model": "scripted", "tools": [WEATHER],
                                             "messages": [{"role": "user", "content": "weather?"}]})
    body = r.json()
    assert r.status_code == 200 and body["choices"][0]["finish_reason"] == "tool_calls"
    msg = body["choices"][0]["message"]
    assert msg["content"] is None and msg["tool_calls"][0]["function"]["name"] == "get_weather"
    assert json.loads(msg["tool_calls"][0]["function"]["arguments"]) == {"city": "Oslo"}
    assert '"name": "get_weather"' in llm.prompts[0]  # the tools went into the prompt


def test_openai_routes_calls_to_gateway_tools_and_continues():
    """execute_tools: the model's calls to example_tool (mock) and vault_tool (secret-gated)
    run through the ToolRouter; their results are fed back and the model's next reply is the
    answer.  Streaming carries the same outcome."""
    from fastapi.testclient import TestClient

    from polykey_service_amd.api.openai import create_app
    call = '<|python_tag|>{"name": "example_tool", "parameters": {}}; {"name": "vault_tool", "parameters": {}}'
    router, llm = _scripted_router([call, "All done."])
    c = TestClient(create_app(router))
    req = {"model": "scripted", "tools": [EXAMPLE, VAULT], "execute_tools": True, "tool_secret_id": "sid-1",
           "messages": [{"role": "user", "content": "run both"}]}
    body = c.post("/v1/chat/completions", json=req).json()
    assert body["choices"][0]["message"] == {"role": "assistant", "content": "All done."}
    assert body["choices"][0]["finish_reason"] == "stop"
    res = body["polykey_tool_results"]
    assert [x["name"] for x in res] == ["example_tool", "vault_tool"]
    assert res[0]["content"].startswith("Mock execution of example_tool at ") and res[0]["status"] == 200
    assert res[1]["content"] == "vault opened with 10-byte key"
    # the second turn saw both results as ipython turns
    assert "ipython<|end_header_id|>\n\nMock execution of example_tool" in llm.prompts[1]
    assert "vault opened with 10-byte key" in llm.prompts[1]
    # without the secret the gated tool reports its error to the model instead of running
    router2, _ = _scripted_router(['{"name": "vault_tool", "parameters": {}}', "no key"])
    body = TestClient(create_app(router2)).post("/v1/chat/completions", json={**req, "tool_secret_id": None}).json()
    assert body["polykey_tool_results"][0]["status"] == "UNAUTHENTICATED"
    # SSE
    router3, _ = _scripted_router(['{"name": "get_weather", "parameters": {"city": "Rome"}}'])
    with TestClient(create_app(router3)).stream("POST", "/v1/chat/completions", json={
            "model": "scripted", "stream": True, "tools": [WEATHER],
            "messages": [{"role": "user", "content": "w"}]}) as resp:
        lines = [json.loads(l[6:]) for l in resp.iter_lines() if l and l != "data: [DONE]"]
    assert lines[0]["choices"][0]["delta"] == {"role": "assistant"}
    tc = lines[1]["choices"][0]["delta"]["tool_calls"][0]
    assert tc["index"] == 0 and tc["function"]["name"] == "get_weather"
    assert lines[-1]["choices"][0]["finish_reason"] == "tool_calls"


def test_grpc_chat_routes_parsed_call():
    router, _ = _scripted_router(['[TOOL_CALLS] [{"name": "struct_tool", "arguments": {}}]', "ok"], MISTRAL)
    tools = [{"type": "function", "function": {"name": "struct_tool"}}]
    with ServerThread(router) as s, grpc.insecure_channel(s.addr) as ch:
        call = ch.unary_unary(proto.EXECUTE_TOOL, request_serializer=proto.ExecuteToolRequest.SerializeToString,
                              response_deserializer=proto.ExecuteToolResponse.FromString)
        req = proto.ExecuteToolRequest(tool_name="llm.chat:scripted")
        req.parameters.update({"messages": [{"role": "user", "content": "go"}], "tools": tools,
                               "execute_tools": True})
        d = proto.struct_to_dict(call(req, timeout=60).struct_output)
    assert d["text"] == "ok" and d["tool_calls"] == []
    res = d["tool_results"][0]
    assert res["name"] == "struct_tool" and json.loads(res["content"])["data"] == {"count": 42.0, "processed": True}


# ------------------------------------------------------------------ real tiny models, forced calls
@pytest.fixture(scope="module")
def model_router():
    r = ToolRouter()
    log = slog.Logger(open("/dev/null", "w"))
    eng = LLMEngine(EngineConfig(model="tiny-mixtral", max_num_seqs=8, max_num_batched_tokens=512, max_model_len=1024,
                                 hip_graphs=False, device="cpu"), ParallelState())
    attach_local_llm(r, ServerConfig(model="tiny-mixtral", backend="local"), log, engine=eng)
    yield r
    r.llm.shutdown()


def test_forced_tool_choice_end_to_end(model_router):
    """A named tool_choice on the random-init Mixtral: the prompt opens the call in Mistral
    format, so the reply is a call to that function whatever the weights; with execute_tools
    the call is routed to the gateway and its outcome fed back before the model answers (random
    weights write no valid JSON arguments, so the routed outcome is the argument error)."""
    from fastapi.testclient import TestClient

    from polykey_service_amd.api.openai import create_app
    assert model_router.llm.tokenizer.chat_template.family == MISTRAL
    c = TestClient(create_app(model_router))
    base = {"model": "tiny-mixtral", "max_tokens": 6, "temperature": 0, "tools": [WEATHER, EXAMPLE],
            "messages": [{"role": "user", "content": "weather?"}]}
    body = c.post("/v1/chat/completions",
                  json={**base, "tool_choice": {"type": "function", "function": {"name": "get_weather"}}}).json()
    assert body["choices"][0]["finish_reason"] == "tool_calls"
    calls = body["choices"][0]["message"]["tool_calls"]
    assert len(calls) == 1 and calls[0]["function"]["name"] == "get_weather"
    assert isinstance(calls[0]["function"]["arguments"], str) and body["usage"]["completion_tokens"] == 6
    body = c.post("/v1/chat/completions", json={**base, "execute_tools": True, "tool_choice": {
        "type": "function", "function": {"name": "example_tool"}}}).json()
    res = body["polykey_tool_results"][0]
    assert res["name"] == "example_tool" and (res["status"] == 400 or res["content"].startswith("Mock execution"))
    assert body["usage"]["completion_tokens"] == 12 and body["choices"][0]["message"]["role"] == "assistant"
    # "required" with one tool forces that tool; "none" renders no tools at all
    body = c.post("/v1/chat/completions", json={**base, "tools": [WEATHER], "tool_choice": "required"}).json()
    assert body["choices"][0]["message"]["tool_calls"][0]["function"]["name"] == "get_weather"
    body = c.post("/v1/chat/completions", json={**base, "tool_choice": "none"}).json()
    assert "tool_calls" not in body["choices"][0]["message"]
    assert c.post("/v1/chat/completions", json={**base, "tool_choice": {"type": "function", "function": {
        "name": "nope"}}}).status_code == 400


def test_forced_tool_choice_grpc(model_router):
    with ServerThread(model_router) as s, grpc.insecure_channel(s.addr) as ch:
        call = ch.unary_unary(proto.EXECUTE_TOOL, request_serializer=proto.ExecuteToolRequest.SerializeToString,
                              response_deserializer=proto.ExecuteToolResponse.FromString)
        req = proto.ExecuteToolRequest(tool_name="llm.chat:tiny-mixtral")
        req.parameters.update({"messages": [{"role": "user", "content": "hi"}], "tools": [WEATHER],
                               "tool_choice": "required", "max_tokens": 4, "temperature": 0})
        d = proto.struct_to_dict(call(req, timeout=60).struct_output)
    assert d["finish_reason"] == "tool_calls" and d["tool_calls"][0]["function"]["name"] == "get_weather"


def test_tool_rounds_are_validated_and_clamped():
    from polykey_service_amd.service import tool_calls
    assert tool_calls.tool_rounds(None) == 3
    assert tool_calls.tool_rounds(2) == 2
    assert tool_calls.tool_rounds(10 ** 6) == tool_calls.MAX_TOOL_ROUNDS
    for bad in (0, -1, "3", 2.5, True, [1]):
        with pytest.raises(ValueError):
            tool_calls.tool_rounds(bad)
