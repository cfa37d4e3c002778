"""Engines of one process on different GPUs: the native ops launch on the calling
thread's current HIP device, so every engine must be BUILT under its device (attach_models,
replicas) and its AsyncLLM thread must BIND its device before the first step."""
import threading

import pytest
import torch

from polykey_service_amd.engine import async_llm


def test_device_guard_and_bind_are_noops_on_cpu():
    with async_llm.device_guard(torch.device("cpu")):
        pass
    with async_llm.device_guard(None):
        pass
    async_llm.bind_device(torch.device("cpu"))
    async_llm.bind_device(None)


def test_engine_thread_binds_the_engine_device(monkeypatch):
    from polykey_service_amd.engine import EngineConfig, LLMEngine
    from polykey_service_amd.parallel.state import ParallelState
    seen = []
    ev = threading.Event()

    def rec(dev):
        seen.append((threading.current_thread().name, dev))
        ev.set()

    monkeypatch.setattr(async_llm, "bind_device", rec)
    eng = LLMEngine(EngineConfig(model="tiny-llama", max_num_seqs=2, max_num_batched_tokens=64, max_model_len=128,
                                 hip_graphs=False, device="cpu"), ParallelState())
    llm = async_llm.AsyncLLM(eng)
    try:
        assert ev.wait(10)
        assert seen[0] == ("polykey-engine", eng.device)
    finally:
        llm.shutdown()


def test_attach_models_builds_each_engine_under_its_device(monkeypatch):
    from polykey_service_amd.adapters import local_llm
    from polykey_service_amd.config.server_config import ServerConfig
    from polykey_service_amd.service import ToolRouter
    from polykey_service_amd.utils import slog
    import io
    import contextlib
    built = []
    real = async_llm.device_guard

    @contextlib.contextmanager
    def rec(dev):
        built.append(str(dev))
        with real(dev):
            yield

    monkeypatch.setattr(async_llm, "device_guard", rec)
    cfg = ServerConfig(backend="local", serve_models="tiny-llama,tiny-mixtral", device="cpu", max_num_seqs=2,
                       max_num_batched_tokens=64, max_model_len=128, hip_graphs=False)
    ms = local_llm.attach_models(ToolRouter(), cfg, slog.Logger(io.StringIO()))
    try:
        assert built == ["cpu", "cpu"]
    finally:
        ms.shutdown()


def test_attach_models_refuses_to_double_book_a_gpu(monkeypatch):
    """An entry without '@' once every GPU is taken: an error, not a silent share of GPU 0."""
    from polykey_service_amd.adapters import local_llm
    from polykey_service_amd.config.server_config import ServerConfig
    from polykey_service_amd.utils import slog
    import io
    monkeypatch.setattr(torch.cuda, "is_available", lambda: True)
    monkeypatch.setattr(torch.cuda, "device_count", lambda: 1)
    cfg = ServerConfig(backend="local", serve_models="tiny-mixtral,tiny-llama@0", device="", max_num_seqs=2)
    with pytest.raises(ValueError, match="no device left"):
        local_llm.attach_models(None, cfg, slog.Logger(io.StringIO()))


def test_decode_workspace_is_sized_for_the_largest_launch():
    """128-key partitions only for launches with < 256 (seq, kv head) workgroups,
    so the slabs hold max(all seqs at 512-key partitions, the few small-launch seqs at 128)."""
    from polykey_service_amd.ops import attention as A
    # Llama-3-8B: 256 seqs, 8 kv heads, 8192 ctx (32-token blocks)
    o, ml = A.decode_workspace(256, 32, 8192 // 32, 32, "cpu", kv_heads=8)
    assert o.shape == (32 * max(256 * 16, 31 * 64), 128) and ml.shape[0] == o.shape[0]
    # 70B TP=8 shard: 1 kv head, 64 seqs, 384 ctx -> all 64 seqs take 128-key partitions
    o, _ = A.decode_workspace(64, 8, 13, 32, "cpu", kv_heads=1)
    assert o.shape[0] == 8 * 64 * 4
    # unknown kv heads: the old conservative size
    o, _ = A.decode_workspace(256, 32, 256, 32, "cpu")
    assert o.shape[0] == 32 * 256 * 64
