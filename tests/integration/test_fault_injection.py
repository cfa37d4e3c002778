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
