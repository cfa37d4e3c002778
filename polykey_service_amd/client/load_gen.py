"""Closed-wave gRPC load generator: the client side of ``bench.py``, run as its own process.

Real clients do not share the server's interpreter; running the 64 concurrent ``ExecuteTool``
clients (request serialisation, response parsing) in the server process made them compete
for the GIL with the engine thread exactly when the engine launches a wave's prefill.  This
process only needs ``grpc`` and the hand-built protobuf schema (no torch, no GPU).

Protocol with the parent over stdin / stdout, one JSON object per line:
    -> {"ready": true}                       warmup waves done, timed requests prebuilt
    <- go
    -> {"tokens": T, "lats": [...], "wall_s": s}

    python -m polykey_service_amd.client.load_gen --addr 127.0.0.1:PORT --tool llm.generate:llama3-8b \\
        --vocab 128256 --concurrency 64 --prompt-len 256 --max-tokens 256 --steps 3 --warmup 1
"""
from __future__ import annotations

import argparse
import asyncio
import json
import os
import random
import sys
import time

import grpc

from .. import proto


def parse_args(argv=None):
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--addr", required=True)
    ap.add_argument("--tool", required=True)
    ap.add_argument("--vocab", type=int, required=True)
    ap.add_argument("--concurrency", type=int, default=64)
    ap.add_argument("--prompt-len", type=int, default=256)
    ap.add_argument("--max-tokens", type=int, default=256)
    ap.add_argument("--mode", choices=["unary", "stream"], default="unary")
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--seed", type=int, default=0)
    return ap.parse_args(argv)


async def run(args) -> dict:
    channel = grpc.aio.insecure_channel(args.addr, options=[
        ("grpc.max_receive_message_length", 64 << 20), ("grpc.max_send_message_length", 64 << 20)])
    unary = channel.unary_unary(proto.EXECUTE_TOOL, request_serializer=proto.ExecuteToolRequest.SerializeToString,
                                response_deserializer=proto.ExecuteToolResponse.FromString)
    stream = channel.unary_stream(proto.EXECUTE_TOOL_STREAM,
                                  request_serializer=proto.ExecuteToolRequest.SerializeToString,
                                  response_deserializer=proto.ExecuteToolResponse.FromString)
    rng = random.Random(args.seed)
    timing = os.environ.get("POLYKEY_BENCH_TIMING") == "1"

    def build():
        req = proto.ExecuteToolRequest(tool_name=args.tool)
        req.parameters.update({"prompt_token_ids": [rng.randrange(0, args.vocab) for _ in range(args.prompt_len)],
                               "max_tokens": args.max_tokens, "ignore_eos": True, "temperature": 0.0,
                               "return": "struct"})
        return req

    async def one(req):
        t0 = time.perf_counter()
        if args.mode == "unary":
            resp = await unary(req, timeout=600)
        else:
            resp = None
            async for resp in stream(req, timeout=600):
                pass
        dt = time.perf_counter() - t0
        usage = resp.struct_output.fields["usage"].struct_value.fields
        return int(usage["completion_tokens"].number_value), dt

    async def wave(reqs):
        tw = time.perf_counter()
        res = await asyncio.gather(*[one(r) for r in reqs])
        if timing:
            print(f"[wave] wall {1e3 * (time.perf_counter() - tw):.1f} ms", file=sys.stderr, flush=True)
        return sum(r[0] for r in res), [r[1] for r in res]

    for _ in range(args.warmup):
        await wave([build() for _ in range(args.concurrency)])
    waves = [[build() for _ in range(args.concurrency)] for _ in range(args.steps)]
    print(json.dumps({"ready": True}), flush=True)
    loop = asyncio.get_running_loop()
    line = await loop.run_in_executor(None, sys.stdin.readline)
    if line.strip() != "go":
        await channel.close()
        return {"error": f"expected 'go', got {line!r}"}
    t0 = time.perf_counter()
    tokens, lats = 0, []
    for reqs in waves:
        n, l = await wave(reqs)
        tokens += n
        lats += l
    wall = time.perf_counter() - t0
    await channel.close()
    return {"tokens": tokens, "lats": lats, "wall_s": wall}


def main(argv=None) -> int:
    out = asyncio.run(run(parse_args(argv)))
    print(json.dumps(out), flush=True)
    return 0 if "error" not in out else 1


if __name__ == "__main__":
    sys.exit(main())
