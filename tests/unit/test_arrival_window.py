"""Arrival coalescing of the async engine loop (engine/async_llm.py): a burst of requests that
lands over a few milliseconds on an idle engine is prefilled in one step, a lone request is
not held back for the whole window, and the window never delays a busy engine."""
import asyncio
import time

import pytest

from polykey_service_amd.engine import EngineConfig, LLMEngine
from polykey_service_amd.engine.async_llm import AsyncLLM
from polykey_service_amd.engine.sequence import SamplingParams
from polykey_service_amd.parallel.state import ParallelState


def _engine(budget=512, max_seqs=16):
    return LLMEngine(EngineConfig(model="tiny-llama", max_num_seqs=max_seqs, max_num_batched_tokens=budget,
                                  max_model_len=512, hip_graphs=False, device="cpu"), ParallelState())


def _record_batches(eng):
    sizes = []
    orig = eng.scheduler.schedule

    def schedule():
        b = orig()
        sizes.append((len(b.prefills), len(b.decodes)))
        return b
    eng.scheduler.schedule = schedule
    return sizes


async def _burst(llm, n, spacing_s, max_tokens=2):
    async def one(i):
        await asyncio.sleep(i * spacing_s)
        return await llm.generate_all(list(range(1, 9)), SamplingParams(max_tokens=max_tokens, ignore_eos=True))
    return await asyncio.gather(*(one(i) for i in range(n)))


@pytest.mark.parametrize("window_ms,expect_one_step", [(60, True), (0, False)])
def test_burst_is_prefilled_together(monkeypatch, window_ms, expect_one_step):
    monkeypatch.setenv("POLYKEY_ARRIVAL_WINDOW_MS", str(window_ms))
    # a gap well above the 1 ms spacing: under a loaded CPU (pytest -n) the client coroutines
    # can run late, and a 5 ms gap once closed the window before the sixth request landed
    monkeypatch.setenv("POLYKEY_ARRIVAL_GAP_MS", "20")
    eng = _engine()
    sizes = _record_batches(eng)
    llm = AsyncLLM(eng)
    try:
        # without a window the burst is spread wider (10 ms) so a loaded CPU cannot merge it by
        # accident before the engine thread wakes for the first request
        outs = asyncio.run(_burst(llm, 6, 0.001 if expect_one_step else 0.01))
    finally:
        llm.shutdown()
    assert all(len(toks) == 2 for toks, _ in outs)
    first = sizes[0][0]
    if expect_one_step:
        assert first == 6, sizes
    else:  # no window: the first request starts alone (the others are still in flight)
        assert first < 6, sizes


def test_lone_request_waits_at_most_one_gap(monkeypatch):
    monkeypatch.setenv("POLYKEY_ARRIVAL_WINDOW_MS", "500")
    monkeypatch.setenv("POLYKEY_ARRIVAL_GAP_MS", "5")
    llm = AsyncLLM(_engine())
    try:
        asyncio.run(_burst(llm, 1, 0.0, max_tokens=1))  # warm-up (first-call overheads)
        t0 = time.perf_counter()
        asyncio.run(_burst(llm, 1, 0.0, max_tokens=1))
        dt = time.perf_counter() - t0
    finally:
        llm.shutdown()
    assert dt < 0.25, f"a lone request was held {dt * 1e3:.0f} ms (window 500 ms, gap 5 ms)"


def test_full_step_is_not_held(monkeypatch):
    """Waiting tokens already fill the budget: the step starts without any wait."""
    eng = _engine(budget=16)
    for i in range(3):
        eng.add_request(list(range(1, 9)), SamplingParams(max_tokens=1), f"r{i}")
    assert not eng.first_step_unfilled()
    eng2 = _engine(budget=512)
    eng2.add_request(list(range(1, 9)), SamplingParams(max_tokens=1), "r")
    assert eng2.first_step_unfilled()
