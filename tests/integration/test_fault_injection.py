"""Fault injection: the engine loop dies mid-stream → open streams fail, health flips to NOT_SERVING."""
import time

import grpc
import pytest

from polykey_service_amd import proto
from polykey_service_amd.adapters.local_llm import attach_local_llm
from polykey_service_amd.config.server_config import ServerConfig
from polykey_service_amd.engine import EngineConfig, LLMEngine
from polykey_service_amd.parallel.state import ParallelState
from polykey_service_amd.server import NOT_SERVING, SERVING
from polykey_service_amd.service import ToolRouter
from polykey_service_amd.utils import slog
from tests.helpers import ServerThread


def test_engine_death_fails_streams_and_health():
    eng = LLMEngine(EngineConfig(model="tiny-llama", max_num_seqs=4, max_num_batched_tokens=64, max_model_len=256,
                                 hip_graphs=False, device="cpu"), ParallelState())
    router = ToolRouter()
    attach_local_llm(router, ServerConfig(model="tiny-llama", backend="local"), slog.Logger(open("/dev/null", "w")),
                     engine=eng)
    real_step = eng.step
    calls = {"n": 0}

    def flaky_step():
        calls["n"] += 1
        if calls["n"] == 4:
            raise RuntimeError("injected HIP fault")
        return real_step()

    eng.step = flaky_step
    with ServerThread(router) as s, grpc.insecure_channel(s.addr) as ch:
        s.loop.call_soon_threadsafe(s.srv.watch_backend, router.llm, 0.05)
        hc = ch.unary_unary(proto.HEALTH_CHECK, request_serializer=proto.HealthCheckRequest.SerializeToString,
                            response_deserializer=proto.HealthCheckResponse.FromString)
        assert hc(proto.HealthCheckRequest(service=""), timeout=5).status == SERVING
        st = ch.unary_stream(proto.EXECUTE_TOOL_STREAM, request_serializer=proto.ExecuteToolRequest.SerializeToString,
                             response_deserializer=proto.ExecuteToolResponse.FromString)
        r = proto.ExecuteToolRequest(tool_name="llm.generate")
        r.parameters.update({"prompt": "boom", "max_tokens": 50, "ignore_eos": True})
        with pytest.raises(grpc.RpcError) as ei:
            list(st(r, timeout=30))
        assert "injected HIP fault" in ei.value.details()
        deadline = time.time() + 5
        while time.time() < deadline and hc(proto.HealthCheckRequest(service=""), timeout=5).status != NOT_SERVING:
            time.sleep(0.05)
        assert hc(proto.HealthCheckRequest(service="polykey.v2.PolykeyService"), timeout=5).status == NOT_SERVING
    router.llm.shutdown()


class _TimedOutAllReduce:
    """Stands in for parallel/custom_ar.CustomAllReduce whose kernel saw a TP peer miss the
    timeout on the 3rd step: ``check`` raises exactly like the host-mapped error word does."""

    def __init__(self, after: int):
        self.after, self.calls = after, 0

    def check(self):
        from polykey_service_amd.parallel.custom_ar import CustomAllReduceError
        self.calls += 1
        if self.calls >= self.after:
            raise CustomAllReduceError("custom all-reduce: a TP peer of rank 0 did not arrive within the timeout")


def test_allreduce_timeout_goes_not_serving_and_exits_nonzero():
    """a TP collective that times out must not produce tokens: the step fails,
    health flips to NOT_SERVING and the server process ends with a non-zero status."""
    import asyncio

    from polykey_service_amd.server import PolykeyServer

    st = ParallelState()
    eng = LLMEngine(EngineConfig(model="tiny-llama", max_num_seqs=4, max_num_batched_tokens=64, max_model_len=256,
                                 hip_graphs=False, device="cpu"), st)
    st.custom_ar = _TimedOutAllReduce(after=3)
    router = ToolRouter()
    attach_local_llm(router, ServerConfig(model="tiny-llama", backend="local"), slog.Logger(open("/dev/null", "w")),
                     engine=eng)

    async def run():
        srv = PolykeyServer(router, slog.Logger(open("/dev/null", "w")), "127.0.0.1:0", own_service=True)
        srv.fatal_grace_s = 0.3
        port = await srv.start()
        srv.watch_backend(router.llm, 0.05)
        serving = asyncio.create_task(srv.serve_until_signal(grace=1.0))
        async with grpc.aio.insecure_channel(f"127.0.0.1:{port}") as ch:
            call = ch.unary_unary(proto.EXECUTE_TOOL, request_serializer=proto.ExecuteToolRequest.SerializeToString,
                                  response_deserializer=proto.ExecuteToolResponse.FromString)
            r = proto.ExecuteToolRequest(tool_name="llm.generate")
            r.parameters.update({"prompt": "x", "max_tokens": 20, "ignore_eos": True})
            with pytest.raises(grpc.aio.AioRpcError) as ei:
                await call(r, timeout=30)
            assert "did not arrive" in ei.value.details()
        statuses = [srv.health.get(proto.POLYKEY_SERVICE)]
        rc = await asyncio.wait_for(serving, timeout=20)
        return rc, statuses

    rc, statuses = asyncio.run(run())
    assert rc == 1
    assert statuses[0] == NOT_SERVING
