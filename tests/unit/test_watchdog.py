"""Step watchdog of the async engine loop (engine/async_llm.py _watch): it judges only a step in
flight, so an engine idle for longer than ``watchdog_s`` serves its next request instead of
declaring itself dead, while a step that really hangs still kills the engine."""
import asyncio
import threading
import time

from polykey_service_amd.engine import EngineConfig, LLMEngine
from polykey_service_amd.engine.async_llm import AsyncLLM, EngineDeadError
from polykey_service_amd.engine.sequence import SamplingParams
from polykey_service_amd.parallel.state import ParallelState


def _engine():
    return LLMEngine(EngineConfig(model="tiny-llama", max_num_seqs=4, max_num_batched_tokens=256,
                                  max_model_len=256, hip_graphs=False, device="cpu"), ParallelState())


def _gen(llm, n=2):
    return asyncio.run(llm.generate_all(list(range(1, 9)), SamplingParams(max_tokens=n, ignore_eos=True)))


def test_idle_longer_than_watchdog_then_submit_is_not_fatal():
    fatal = []
    eng = _engine()
    # the first step after the idle gap runs longer than the watchdog's 0.5 s poll period, so
    # a watchdog that measured from the last *finished* step would certainly fire inside it
    orig = eng.step
    slow = [False]

    def step():
        if slow[0]:
            slow[0] = False
            time.sleep(0.6)
        return orig()
    eng.step = step
    llm = AsyncLLM(eng, on_fatal=fatal.append, watchdog_s=1.0)
    try:
        _gen(llm)
        time.sleep(2.2)  # idle for twice the watchdog period
        assert llm.healthy()
        slow[0] = True
        toks, _ = _gen(llm, 4)
        assert len(toks) == 4
        time.sleep(0.6)  # the watchdog polled again after the request
    finally:
        llm.shutdown()
    assert not fatal and llm.dead is None


def test_hung_step_is_fatal():
    fatal = []
    eng = _engine()
    release = threading.Event()
    orig = eng.step

    def hung_step():
        release.wait(10.0)
        return orig()
    eng.step = hung_step
    eng.runner.abort_comms = lambda: release.set()  # the watchdog aborts the "collective"
    llm = AsyncLLM(eng, on_fatal=fatal.append, watchdog_s=0.3)
    try:
        t0 = time.monotonic()
        try:
            _gen(llm)
            raised = False
        except EngineDeadError:
            raised = True
        assert raised and time.monotonic() - t0 < 5.0
        assert not llm.healthy()
    finally:
        release.set()
        llm.shutdown()
    assert len(fatal) == 1 and isinstance(fatal[0], TimeoutError)
