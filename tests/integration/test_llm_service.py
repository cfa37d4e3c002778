"""LLM tools end to end on CPU (tiny Llama/Mixtral, reference ops): gRPC unary + streaming,
cancellation frees KV, OpenAI-compatible HTTP route, model routing (config 5 tool-call path)."""
import asyncio
import json
import threading
import time

import grpc
import pytest

from polykey_service_amd import proto
from polykey_service_amd.adapters.local_llm import LLMTool, attach_local_llm
from polykey_service_amd.config.server_config import ServerConfig
from polykey_service_amd.engine import EngineConfig, LLMEngine
from polykey_service_amd.engine.async_llm import AsyncLLM
from polykey_service_amd.engine.sequence import SamplingParams
from polykey_service_amd.parallel.state import ParallelState
from polykey_service_amd.service import ToolRouter
from polykey_service_amd.utils import slog

from tests.helpers import ServerThread


def make_engine(model="tiny-llama", **kw):
    return LLMEngine(EngineConfig(model=model, max_num_seqs=8, max_num_batched_tokens=128, max_model_len=512,
                                  hip_graphs=False, device="cpu", **kw), ParallelState())


@pytest.fixture(scope="module")
def router():
    r = ToolRouter()
    log = slog.Logger(open("/dev/null", "w"))
    attach_local_llm(r, ServerConfig(model="tiny-llama", backend="local"), log, engine=make_engine())
    # a second backend to exercise model routing ("llm.chat:<model>")
    mix = AsyncLLM(make_engine("tiny-mixtral"))
    r.register_model_tool("llm.chat", "tiny-mixtral", LLMTool("llm.chat", "tiny-mixtral", mix, chat=True))
    r.register_model_tool("llm.generate", "tiny-mixtral", LLMTool("llm.generate", "tiny-mixtral", mix, chat=False))
    yield r
    r.llm.shutdown()
    mix.shutdown()


def req(tool, **params):
    r = proto.ExecuteToolRequest(tool_name=tool)
    r.parameters.update(params)
    return r


def test_unary_generate_text_and_struct(router):
    with ServerThread(router) as s, grpc.insecure_channel(s.addr) as ch:
        call = ch.unary_unary(proto.EXECUTE_TOOL, request_serializer=proto.ExecuteToolRequest.SerializeToString,
                              response_deserializer=proto.ExecuteToolResponse.FromString)
        r = call(req("llm.generate", prompt="hello", max_tokens=5, ignore_eos=True), timeout=60)
        assert r.status.code == 200 and r.WhichOneof("output") == "string_output"
        r = call(req("llm.generate", prompt_token_ids=[1, 5, 6], max_tokens=7, ignore_eos=True, **{"return": "struct"}),
                 timeout=60)
        d = proto.struct_to_dict(r.struct_output)
        assert d["usage"] == {"prompt_tokens": 3.0, "completion_tokens": 7.0, "total_tokens": 10.0}
        assert d["finish_reason"] == "length" and d["model"] == "tiny-llama"
        # mock tools still behave exactly like the reference next to the model tools
        assert call(req("example_tool"), timeout=5).string_output.startswith("Mock execution of example_tool at ")
        with pytest.raises(grpc.RpcError) as ei:
            call(req("llm.generate", max_tokens=3), timeout=10)
        assert ei.value.code() == grpc.StatusCode.INVALID_ARGUMENT


def test_greedy_is_deterministic_and_batch_invariant(router):
    with ServerThread(router) as s, grpc.insecure_channel(s.addr) as ch:
        call = ch.unary_unary(proto.EXECUTE_TOOL, request_serializer=proto.ExecuteToolRequest.SerializeToString,
                              response_deserializer=proto.ExecuteToolResponse.FromString)
        one = call(req("llm.generate", prompt="same prompt", max_tokens=8, ignore_eos=True), timeout=60).string_output
        futs = [call.future(req("llm.generate", prompt="same prompt", max_tokens=8, ignore_eos=True), timeout=60)
                for _ in range(6)]
        assert all(f.result().string_output == one for f in futs)


def test_streaming_chunks_and_final_usage(router):
    with ServerThread(router) as s, grpc.insecure_channel(s.addr) as ch:
        st = ch.unary_stream(proto.EXECUTE_TOOL_STREAM, request_serializer=proto.ExecuteToolRequest.SerializeToString,
                             response_deserializer=proto.ExecuteToolResponse.FromString)
        chunks = list(st(req("llm.chat", messages=[{"role": "user", "content": "hi"}], max_tokens=12,
                             ignore_eos=True), timeout=60))
        assert len(chunks) >= 2
        final = proto.struct_to_dict(chunks[-1].struct_output)
        text = "".join(c.string_output for c in chunks[:-1])
        assert final["usage"]["completion_tokens"] == 12 and final["text"] == text
        assert chunks[-1].status.code == 200


def test_model_routing_to_mixtral(router):
    with ServerThread(router) as s, grpc.insecure_channel(s.addr) as ch:
        call = ch.unary_unary(proto.EXECUTE_TOOL, request_serializer=proto.ExecuteToolRequest.SerializeToString,
                              response_deserializer=proto.ExecuteToolResponse.FromString)
        r = call(req("llm.chat:tiny-mixtral", messages=[{"role": "user", "content": "route me"}], max_tokens=4,
                     ignore_eos=True, **{"return": "struct"}), timeout=60)
        assert proto.struct_to_dict(r.struct_output)["model"] == "tiny-mixtral"
        with pytest.raises(grpc.RpcError) as ei:
            call(req("llm.chat:nope", messages=[{"role": "user", "content": "x"}]), timeout=10)
        assert ei.value.code() == grpc.StatusCode.NOT_FOUND


def test_cancellation_frees_kv(router):
    eng = router.llm.engine
    free0 = eng.bm.num_free
    with ServerThread(router) as s, grpc.insecure_channel(s.addr) as ch:
        st = ch.unary_stream(proto.EXECUTE_TOOL_STREAM, request_serializer=proto.ExecuteToolRequest.SerializeToString,
                             response_deserializer=proto.ExecuteToolResponse.FromString)
        it = st(req("llm.generate", prompt="long " * 20, max_tokens=400, ignore_eos=True), timeout=60)
        next(it)
        it.cancel()
        deadline = time.time() + 20
        while time.time() < deadline and (eng.has_unfinished() or eng.bm.num_free != free0):
            time.sleep(0.05)
    assert not eng.has_unfinished() and eng.bm.num_free == free0


def test_concurrent_streams_interleave(router):
    async def run():
        async with grpc.aio.insecure_channel(addr) as ch:
            st = ch.unary_stream(proto.EXECUTE_TOOL_STREAM,
                                 request_serializer=proto.ExecuteToolRequest.SerializeToString,
                                 response_deserializer=proto.ExecuteToolResponse.FromString)

            async def one(i):
                n = 0
                async for c in st(req("llm.generate", prompt_token_ids=[1, 3 + i], max_tokens=6, ignore_eos=True),
                                  timeout=60):
                    if c.HasField("struct_output"):
                        n = int(c.struct_output["usage"]["completion_tokens"])
                return n

            return await asyncio.gather(*[one(i) for i in range(16)])

    with ServerThread(router) as s:
        addr = s.addr
        assert asyncio.run(run()) == [6] * 16


def test_openai_routes(router):
    from fastapi.testclient import TestClient

    from polykey_service_amd.api.openai import create_app
    c = TestClient(create_app(router))
    assert c.get("/health").json() == {"status": "ok"}
    models = [m["id"] for m in c.get("/v1/models").json()["data"]]
    assert "tiny-llama" in models and "tiny-mixtral" in models
    r = c.post("/v1/chat/completions", json={"model": "tiny-llama", "max_tokens": 5, "ignore_eos": True,
                                             "temperature": 0, "messages": [{"role": "user", "content": "hey"}]})
    body = r.json()
    assert r.status_code == 200 and body["object"] == "chat.completion"
    assert body["usage"]["completion_tokens"] == 5 and body["choices"][0]["message"]["role"] == "assistant"
    r = c.post("/v1/completions", json={"model": "tiny-llama", "prompt": [1, 4, 5], "max_tokens": 3,
                                        "ignore_eos": True})
    assert r.json()["usage"] == {"prompt_tokens": 3, "completion_tokens": 3, "total_tokens": 6,
                                 "prompt_tokens_details": {"cached_tokens": 0}}
    # the same 70-token prompt again: its first two 32-token KV blocks come from the prefix cache
    long_prompt = [1] + list(range(500, 569))
    for cached in (0, 64):
        r = c.post("/v1/completions", json={"model": "tiny-llama", "prompt": long_prompt, "max_tokens": 2,
                                            "ignore_eos": True})
        assert r.json()["usage"]["prompt_tokens_details"]["cached_tokens"] == cached
    with c.stream("POST", "/v1/chat/completions", json={"model": "tiny-llama", "stream": True, "max_tokens": 6,
                                                        "ignore_eos": True,
                                                        "messages": [{"role": "user", "content": "s"}]}) as resp:
        lines = [l for l in resp.iter_lines() if l]
    assert lines[-1] == "data: [DONE]"
    last = json.loads(lines[-2][len("data: "):])
    assert last["usage"]["completion_tokens"] == 6 and last["choices"][0]["finish_reason"] == "length"
    assert c.post("/v1/chat/completions", json={"model": "nope", "messages": [{"role": "user", "content": "x"}]}
                  ).status_code == 404
    assert c.post("/v1/chat/completions", json={"messages": []}).status_code == 400


def test_replica_pool_balances_requests():
    from polykey_service_amd.adapters.local_llm import ReplicaPool
    pool = ReplicaPool([AsyncLLM(make_engine()), AsyncLLM(make_engine())])
    r = ToolRouter()
    r.register_model_tool("llm.generate", "tiny-llama", LLMTool("llm.generate", "tiny-llama", pool, chat=False))
    r.llm = pool

    async def run():
        async with grpc.aio.insecure_channel(addr) as ch:
            call = ch.unary_unary(proto.EXECUTE_TOOL, request_serializer=proto.ExecuteToolRequest.SerializeToString,
                                  response_deserializer=proto.ExecuteToolResponse.FromString)
            outs = await asyncio.gather(*[call(req("llm.generate", prompt="balance", max_tokens=6, ignore_eos=True),
                                               timeout=60) for _ in range(12)])
            return [o.string_output for o in outs]

    with ServerThread(r) as s:
        addr = s.addr
        outs = asyncio.run(run())
    assert len(set(outs)) == 1  # same weights (same seed) on both replicas → same greedy text
    assert all(rep.stats["requests"] > 0 for rep in pool.replicas)
    pool.shutdown()


def test_torch_profiler_toggle(tmp_path, monkeypatch):
    """POLYKEY_TORCH_PROFILE=<dir> records a Chrome trace of engine steps."""
    monkeypatch.setenv("POLYKEY_TORCH_PROFILE", str(tmp_path))
    llm = AsyncLLM(make_engine())

    async def run():
        return await llm.generate_all([1, 5, 6, 7], SamplingParams(max_tokens=60, ignore_eos=True))

    toks, last = asyncio.run(run())
    llm.shutdown()
    assert len(toks) == 60 and last.finished
    assert any(p.name.endswith(".json") or p.name.endswith(".json.gz") for p in tmp_path.iterdir())


def test_serve_models_routes_one_front_end_to_several_engines():
    """``serve_models`` (POLYKEY_SERVE_MODELS): one gRPC front end, two models, each on its own
    engine (its own device on a GPU node); ``<family>:<model>`` routes to each, the first listed
    is the default, health follows every engine, an unknown model is NOT_FOUND."""
    from polykey_service_amd.adapters.local_llm import ModelSet, parse_serve_models
    from polykey_service_amd.server.app import build_service

    assert parse_serve_models("llama3-8b@0-3,mixtral-8x7b@4,x") == [
        ("llama3-8b", [0, 1, 2, 3]), ("mixtral-8x7b", [4]), ("x", [])]
    with pytest.raises(ValueError):
        parse_serve_models("a@0,a@1")
    cfg = ServerConfig(backend="local", serve_models="tiny-llama,tiny-mixtral", device="cpu", max_num_seqs=8,
                       max_num_batched_tokens=128, max_model_len=512, hip_graphs=False)
    router = build_service(cfg, slog.Logger(open("/dev/null", "w")))
    try:
        assert isinstance(router.llm, ModelSet) and sorted(router.llm.llms) == ["tiny-llama", "tiny-mixtral"]
        assert router.models("llm.chat") == ["tiny-llama", "tiny-mixtral"] and router.llm.healthy()
        engines = {n: getattr(l, "engine", None) for n, l in router.llm.llms.items()}
        assert engines["tiny-llama"] is not engines["tiny-mixtral"]
        with ServerThread(router) as s, grpc.insecure_channel(s.addr) as ch:
            call = ch.unary_unary(proto.EXECUTE_TOOL, request_serializer=proto.ExecuteToolRequest.SerializeToString,
                                  response_deserializer=proto.ExecuteToolResponse.FromString)
            for tool, want in (("llm.generate:tiny-llama", "tiny-llama"), ("llm.generate:tiny-mixtral", "tiny-mixtral"),
                               ("llm.generate", "tiny-llama")):
                r = call(req(tool, prompt_token_ids=[1, 5, 6], max_tokens=3, ignore_eos=True, **{"return": "struct"}),
                         timeout=60)
                d = proto.struct_to_dict(r.struct_output)
                assert d["model"] == want and d["usage"]["completion_tokens"] == 3.0, (tool, d)
            r = call(req("llm.chat:tiny-mixtral", messages=[{"role": "user", "content": "hi"}], max_tokens=2,
                         ignore_eos=True), timeout=60)
            assert r.status.code == 200
            with pytest.raises(grpc.RpcError) as ei:
                call(req("llm.generate:no-such-model", prompt="x", max_tokens=1), timeout=10)
            assert ei.value.code() == grpc.StatusCode.NOT_FOUND
    finally:
        router.llm.shutdown()
