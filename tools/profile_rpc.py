"""Host cost of the gRPC path of bench.py with the engine stubbed out (CPU only): one asyncio
loop serves ``polykey.v2.PolykeyService`` and drives 64 concurrent ExecuteTool clients, each
sending 256 prompt token ids and receiving a 256-token struct summary, exactly as bench.py
does.  Prints per-wave wall time and a cProfile of the loop.

    python tools/profile_rpc.py [waves] [concurrency]
"""
import asyncio
import cProfile
import os
import pstats
import random
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import grpc  # noqa: E402

from polykey_service_amd import proto  # noqa: E402
from polykey_service_amd.adapters.local_llm import LLMTool  # noqa: E402
from polykey_service_amd.engine.sequence import RequestOutput  # noqa: E402
from polykey_service_amd.engine.tokenizer import get_tokenizer  # noqa: E402
from polykey_service_amd.server import PolykeyServer  # noqa: E402
from polykey_service_amd.service import ToolRouter  # noqa: E402
from polykey_service_amd.utils import slog  # noqa: E402


class StubLLM:
    """Duck-types AsyncLLM.generate: the whole completion in one RequestOutput."""

    def __init__(self):
        self.tokenizer = get_tokenizer("", 128256, 128000, 128001)

    async def generate(self, prompt_ids, params, request_id=None, final_only=False):
        yield RequestOutput(request_id or "r", list(range(params.max_tokens)), True, "length", len(prompt_ids),
                            params.max_tokens, {"queue_s": 0.0, "ttft_s": 0.0, "e2e_s": 0.0})


async def main(waves: int, conc: int):
    logger = slog.Logger(open(os.devnull, "w"))
    router = ToolRouter()
    llm = StubLLM()
    router.register_model_tool("llm.generate", "llama3-8b", LLMTool("llm.generate", "llama3-8b", llm, chat=False))
    srv = PolykeyServer(router, logger, "127.0.0.1:0", own_service=False)
    port = await srv.start()
    ch = grpc.aio.insecure_channel(f"127.0.0.1:{port}")
    unary = ch.unary_unary(proto.EXECUTE_TOOL, request_serializer=proto.ExecuteToolRequest.SerializeToString,
                           response_deserializer=proto.ExecuteToolResponse.FromString)
    rng = random.Random(0)

    def build():
        req = proto.ExecuteToolRequest(tool_name="llm.generate:llama3-8b")
        req.parameters.update({"prompt_token_ids": [rng.randrange(0, 128256) for _ in range(256)],
                               "max_tokens": 256, "ignore_eos": True, "temperature": 0.0, "return": "struct"})
        return req

    async def one(req=None):
        r = await unary(req or build(), timeout=60)
        assert r.status.code == 200

    await asyncio.gather(*[one() for _ in range(conc)])  # warm up
    pr = cProfile.Profile()
    pr.enable()
    for _ in range(waves):
        reqs = [build() for _ in range(conc)]  # prebuilt, as bench.py does
        t0 = time.perf_counter()
        await asyncio.gather(*[one(r) for r in reqs])
        print(f"wave of {conc}: {1e3 * (time.perf_counter() - t0):.1f} ms", flush=True)
    pr.disable()
    await ch.close()
    await srv.stop(0)
    pstats.Stats(pr).sort_stats("tottime").print_stats(25)


if __name__ == "__main__":
    asyncio.run(main(int(sys.argv[1]) if len(sys.argv) > 1 else 3, int(sys.argv[2]) if len(sys.argv) > 2 else 64))
