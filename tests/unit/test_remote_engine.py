"""Front end <-> engine process protocol (engine/remote.py) on the CPU: a RemoteEngine handle
served by an EngineServer over a local socket returns the same greedy tokens as the engine
called in-process, streams per step or reports once (final_only), aborts free the engine's
KV, the least-loaded router spreads requests, and a vanished engine fails its requests."""
import asyncio
import threading

import pytest

from polykey_service_amd.adapters.local_llm import ReplicaPool
from polykey_service_amd.engine import EngineConfig, LLMEngine
from polykey_service_amd.engine.async_llm import AsyncLLM
from polykey_service_amd.engine.remote import EngineServer, RemoteEngine
from polykey_service_amd.engine.sequence import SamplingParams
from polykey_service_amd.parallel.state import ParallelState


def _llm():
    eng = LLMEngine(EngineConfig(model="tiny-llama", max_num_seqs=8, max_num_batched_tokens=256, max_model_len=512,
                                 hip_graphs=False, device="cpu"), ParallelState())
    return AsyncLLM(eng)


@pytest.fixture()
def served():
    llm = _llm()
    srv = EngineServer(llm)
    th = threading.Thread(target=srv.serve, daemon=True)
    th.start()
    remote = RemoteEngine(("127.0.0.1", srv.port), llm.tokenizer, name="t")
    remote.server = srv  # for tests that inspect the engine side
    yield llm, remote
    remote.shutdown()
    th.join(10)
    assert not th.is_alive()
    llm.shutdown()


PROMPT = [3, 1, 4, 1, 5, 9, 2, 6]


def test_remote_matches_local_and_streams(served):
    llm, remote = served
    sp = SamplingParams(max_tokens=6, ignore_eos=True)

    async def go():
        local, _ = await llm.generate_all(PROMPT, sp)
        rtoks, last = await remote.generate_all(PROMPT, sp)
        chunks = [o async for o in remote.generate(PROMPT, sp)]
        finals = [o async for o in remote.generate(PROMPT, sp, final_only=True)]
        return local, rtoks, last, chunks, finals
    local, rtoks, last, chunks, finals = asyncio.run(go())
    assert rtoks == local and len(rtoks) == 6
    assert last.finished and last.num_output_tokens == 6 and last.num_prompt_tokens == len(PROMPT)
    assert len(chunks) > 1 and sum((c.new_token_ids for c in chunks), []) == local
    assert len(finals) == 1 and finals[0].new_token_ids == local


def test_abort_frees_engine_state(served):
    llm, remote = served

    async def go():
        agen = remote.generate(PROMPT, SamplingParams(max_tokens=200, ignore_eos=True))
        first = await agen.__anext__()
        await agen.aclose()  # client went away -> abort frame
        for _ in range(200):
            if not llm.engine.has_unfinished():
                break
            await asyncio.sleep(0.01)
        return first
    first = asyncio.run(go())
    assert first.new_token_ids
    assert not llm.engine.has_unfinished()
    assert llm.engine.bm.num_free == llm.engine.runner.num_blocks


def test_pool_routes_to_least_loaded(served):
    llm, remote = served
    pool = ReplicaPool([llm, remote])
    sp = SamplingParams(max_tokens=4, ignore_eos=True)

    async def go():
        return await asyncio.gather(*(pool.generate_all(PROMPT, sp) for _ in range(6)))
    outs = asyncio.run(go())
    assert all(t == outs[0][0] for t, _ in outs)
    assert llm.stats["requests"] >= 6  # remote requests run on the served engine too


def test_dead_engine_fails_requests():
    llm = _llm()
    srv = EngineServer(llm)
    th = threading.Thread(target=srv.serve, daemon=True)
    th.start()
    remote = RemoteEngine(("127.0.0.1", srv.port), llm.tokenizer, name="d")
    remote.sock.shutdown(2)  # the connection dies under the front end
    th.join(10)
    remote._reader.join(10)
    assert not remote.healthy()

    async def go():
        with pytest.raises(RuntimeError):
            await remote.generate_all(PROMPT, SamplingParams(max_tokens=2))
    asyncio.run(go())
    remote.shutdown()
    llm.shutdown()


def test_engine_server_rejects_a_front_end_without_the_token():
    """The engine server serves only the front end presenting the shared token (dp_gateway draws
    it on rank 0); an unauthenticated connection is closed and the server keeps listening."""
    import socket as _socket
    llm = _llm()
    srv = EngineServer(llm, token="s3cret")
    th = threading.Thread(target=srv.serve, daemon=True)
    th.start()
    intruder = _socket.create_connection(("127.0.0.1", srv.port))
    intruder.sendall(b"\x05\x00\x00\x00hello")  # not a valid hello frame
    intruder.settimeout(10)
    assert intruder.recv(16) == b""  # closed by the server
    intruder.close()
    remote = RemoteEngine(("127.0.0.1", srv.port), llm.tokenizer, name="t", token="s3cret")
    sp = SamplingParams(max_tokens=3, ignore_eos=True)
    toks, _ = asyncio.run(remote.generate_all(PROMPT, sp))
    assert len(toks) == 3
    remote.shutdown()
    th.join(10)
    llm.shutdown()


def test_abort_of_a_final_only_request_drops_its_buffer(served):
    llm, remote = served

    async def go():
        agen = remote.generate(PROMPT, SamplingParams(max_tokens=200, ignore_eos=True), request_id="r-final",
                               final_only=True)
        task = asyncio.ensure_future(agen.__anext__())
        await asyncio.sleep(0.3)
        task.cancel()
        try:
            await task
        except (asyncio.CancelledError, StopAsyncIteration):
            pass
        await agen.aclose()
    asyncio.run(go())
    import time as _t
    deadline = _t.monotonic() + 5
    servers = [remote.server]
    while _t.monotonic() < deadline and any("r-final" in s._final for s in servers):
        _t.sleep(0.05)
    assert not any("r-final" in s._final for s in servers)
