#!/usr/bin/env python
"""Headline benchmark: output tokens/s via gRPC (+ p50 E2E latency), Llama-3-8B bf16.

Metric/config from BASELINE.json ("output tokens/sec via gRPC + p50 E2E latency, Llama-3-8B
TP=1 / 70B TP=8").  One process per GPU (torchrun); with ``--tp 1`` every rank is an
independent Llama-3-8B replica (request-level data parallel → weak scaling: per-GPU work is
fixed as N grows) that serves a real ``polykey.v2.PolykeyService`` gRPC server on
127.0.0.1 and is driven by ``--concurrency`` concurrent ``ExecuteTool`` clients in the same
process.  With ``--tp 8 --model llama3-70b`` the 8 ranks form one tensor-parallel replica
(RCCL all-reduce over xGMI) and rank 0 serves the gRPC endpoint.  The clients run in a load
generator process of their own per replica with ``--client process``
(``polykey_service_amd.client.load_gen``); by default they run on the server's event loop.

A "step" is one wave of ``--concurrency`` requests per replica, each a synthetic
``--prompt-len``-token prompt generating exactly ``--max-tokens`` tokens (``ignore_eos``,
random-init weights, synthetic token ids — no network for checkpoints/datasets).
W warmup waves run untimed; then K waves are timed between a barrier + device sync on both
sides; elapsed = max over ranks; value = total output tokens of all replicas / elapsed.

    python bench.py --gpus N --steps K --warmup W
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 bench.py --gpus N ...

With N > 1 (plain, or rank 0 of the driver's torchrun -- the other outer ranks exit without
touching a GPU) the measurement runs in a fresh N-rank torchrun child whose JSON line is relayed;
with ``--tp 1`` a second child then serves ``--tp-extra-model`` (default Llama-3-70B) at TP = N
over the same gRPC load and its result is added under ``tp{N}_70b`` -- the 70B TP=8 half of the
BASELINE metric on an 8-GPU node -- and a third child serves ``--ep-extra-model`` (default
Mixtral-8x7B) with DP attention + expert parallelism over all N GPUs (IPC expert all-to-all),
reported under ``ep{N}_mixtral`` (BASELINE config 5).  Each child has its own timeout inside ONE
deadline: an extra child's failure is reported in its key and never loses the replica number.
"""
from __future__ import annotations

import argparse
import asyncio
import json
import os
import random
import statistics
import subprocess
import sys
import time

METRIC = "output tokens/sec via gRPC + p50 E2E latency, Llama-3-8B TP=1 / 70B TP=8"
MODEL_NAMES = {"llama3-8b": "Llama-3-8B", "llama3-70b": "Llama-3-70B", "mixtral-8x7b": "Mixtral-8x7B"}


def parse_args(argv=None):
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--model", default="llama3-8b")
    ap.add_argument("--tp", type=int, default=1)
    ap.add_argument("--ep", type=int, default=1,
                    help="expert parallel degree (MoE): = --tp for EP inside the TP group, or = --gpus with "
                         "--tp 1 for DP attention + expert all-to-all")
    ap.add_argument("--concurrency", type=int, default=64, help="concurrent gRPC clients per replica")
    ap.add_argument("--prompt-len", type=int, default=256)
    ap.add_argument("--max-tokens", type=int, default=256)
    ap.add_argument("--mode", choices=["unary", "stream", "openai"], default="unary",
                    help="unary / server-streaming ExecuteTool over gRPC, or POST /v1/chat/completions on the "
                         "OpenAI-compatible route (api/openai.py) served by the same process")
    ap.add_argument("--max-batched-tokens", type=int, default=8192)
    ap.add_argument("--no-graphs", action="store_true")
    ap.add_argument("--num-kv-blocks", type=int, default=0, help="KV blocks per replica (0: size from free HBM)")
    ap.add_argument("--gpu-mem-fraction", type=float, default=0.90)
    ap.add_argument("--port-base", type=int, default=int(os.environ.get("POLYKEY_BENCH_PORT", "0")),
                    help="gRPC port of rank 0 (rank r: base + r); 0: an ephemeral port per rank")
    ap.add_argument("--seed", type=int, default=0)
    # measured on 1x MI355X (profiles/r2_bench_client_ab.txt): unary 12,879 tok/s with the clients on
    # the server's event loop vs 12,299 from a separate load-generator process (streaming: 12,787)
    ap.add_argument("--frontend", choices=["replicas", "single"], default="replicas",
                    help="N > 1, tp 1: every rank serves its own gRPC endpoint (replicas, the DP design); or rank 0 "
                         "alone as the front end, routing to every rank's engine process (single, "
                         "engine/remote.py dp_gateway)")
    ap.add_argument("--client", choices=["process", "inproc"], default="inproc",
                    help="load generator on the server's event loop (default) or in its own process")
    ap.add_argument("--tp-extra-model", default="auto",
                    help="N > 1 with --tp 1: after the replica run, measure this model at TP = N in a fresh "
                         "torchrun child and report it under the extra key tp{N}_<model> (BASELINE.json: "
                         "'Llama-3-8B TP=1 / 70B TP=8'); auto: llama3-70b when --model is llama3-8b (the "
                         "BASELINE pair), else none; 'none' skips it")
    ap.add_argument("--tp-extra-mode", choices=["unary", "stream", "openai"], default="openai",
                    help="the TP child's request path: BASELINE config 4 is '70B TP=8 over xGMI, OpenAI-compatible "
                         "chat route'")
    ap.add_argument("--tp-extra-timeout", type=float, default=480.0,
                    help="seconds the TP child may take at most (its failure or timeout never loses the main number)")
    ap.add_argument("--ep-extra-model", default="auto",
                    help="N > 1 with --tp 1: after the TP child, measure this MoE model with DP attention + EP = N "
                         "(expert all-to-all over all N GPUs) under ep{N}_<model> (BASELINE config 5); auto: "
                         "mixtral-8x7b when --model is llama3-8b and N divides its experts, else none")
    ap.add_argument("--extra-steps", type=int, default=5,
                    help="timed waves of the tp{N} / ep{N} children (at most --steps)")
    ap.add_argument("--ep-extra-timeout", type=float, default=300.0,
                    help="seconds the EP child may take at most (never at the main number's expense)")
    ap.add_argument("--child-timeout", type=float, default=1500.0, help="seconds the main measurement child may take")
    ap.add_argument("--deadline", type=float, default=float(os.environ.get("POLYKEY_BENCH_DEADLINE_S", "540")),
                    help="N > 1: seconds the whole run may take, below the driver's 600 s command limit. The main "
                         "child gets at most this minus a print margin, the TP child only what is left, so the "
                         "JSON line is always printed in time")
    ap.add_argument("--child", action="store_true", help=argparse.SUPPRESS)  # internal: the measuring torchrun job
    return ap.parse_args(argv)


# torchrun's per-worker variables: a nested launch must not inherit the outer job's rendezvous
_LAUNCH_ENV = ("RANK", "LOCAL_RANK", "WORLD_SIZE", "LOCAL_WORLD_SIZE", "GROUP_RANK", "GROUP_WORLD_SIZE",
               "ROLE_RANK", "ROLE_WORLD_SIZE", "ROLE_NAME", "MASTER_ADDR", "MASTER_PORT")


def _free_port() -> int:
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def kill_tree(p: "subprocess.Popen") -> None:
    """SIGKILL ``p``, its process group and every descendant.  torchrun's ranks run in sessions
    of their own: killing the launcher's group alone orphans them -- they keep the stdout pipe
    open (so a ``communicate`` after the kill never sees EOF) and, hung, never exit."""
    import signal
    try:
        import psutil
        kids = psutil.Process(p.pid).children(recursive=True)
    except Exception:  # psutil missing or the launcher already gone
        kids = []
    try:
        os.killpg(p.pid, signal.SIGKILL)
    except (ProcessLookupError, PermissionError):
        pass
    for k in kids:
        try:
            k.kill()
        except Exception:
            pass


def run_child(argv, n: int, timeout: float):
    """One measurement as a fresh torchrun job of ``n`` ranks (a child process, never an exec;
    its own session, so a timeout kills the whole tree and frees every GPU).  Returns
    (rc, the child's JSON line as a dict or None, wall seconds)."""
    env = {k: v for k, v in os.environ.items() if k not in _LAUNCH_ENV and not k.startswith("TORCHELASTIC_")}
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.abspath(__file__)] + argv
    t0 = time.perf_counter()
    p = subprocess.Popen(cmd, env=env, stdout=subprocess.PIPE, text=True, start_new_session=True)
    try:
        out, _ = p.communicate(timeout=timeout)
        rc = p.returncode
    except subprocess.TimeoutExpired:
        kill_tree(p)
        try:
            out, _ = p.communicate(timeout=30)
        except subprocess.TimeoutExpired:  # a descendant that escaped still holds the pipe
            out = ""
        rc = 124
    line = None
    for ln in out.splitlines():
        if ln.startswith("{"):
            try:
                line = json.loads(ln)
            except ValueError:
                pass
        else:
            print(ln, file=sys.stderr)
    return rc, line, time.perf_counter() - t0


def _strip(argv, names):
    """argv without the options in ``names`` (and their values)."""
    out, skip = [], False
    for a in argv:
        if skip:
            skip = False
            continue
        k = a.split("=", 1)[0]
        if k in names:
            skip = "=" not in a
            continue
        out.append(a)
    return out


def _extra_key(prefix: str, n: int, model: str) -> str:
    return f"{prefix}{n}_" + {"llama3-70b": "70b", "llama3-8b": "8b", "mixtral-8x7b": "mixtral"}.get(model, model)


def orchestrate(args, argv) -> int:
    """``--gpus N`` (N > 1), plain or under the driver's torchrun (rank 0 only: the other outer
    ranks exit without touching a GPU).  The measurement runs as a fresh N-rank torchrun child
    whose JSON line is relayed; with ``--tp 1`` two more children then measure the other BASELINE
    configs on the same N GPUs: ``--tp-extra-model`` at TP = N (70B TP=8 on an 8-GPU node) under
    ``tp{N}_<model>`` and ``--ep-extra-model`` with DP attention + EP = N (Mixtral expert
    all-to-all) under ``ep{N}_<model>``.  Each child has its own timeout, so an extra child's
    failure can never erase the replica number, and all of them live inside ONE ``--deadline``:
    a later child gets only what the earlier ones left (a hung child is killed in time for the
    line to be printed before the driver's own limit)."""
    t_start = time.monotonic()

    def left() -> float:  # seconds a child may still take, keeping a margin to print the line
        return args.deadline - (time.monotonic() - t_start) - 10.0

    rc, main_line, _ = run_child(argv + ["--child"], args.gpus, max(1.0, min(args.child_timeout, left())))
    if main_line is None:
        print(f"bench: measurement child failed (rc {rc})", file=sys.stderr)
        return rc or 1
    strip = {"--model", "--tp", "--ep", "--frontend", "--tp-extra-model", "--ep-extra-model", "--mode",
             "--tp-extra-mode"}

    def extra_child(key: str, cargs, timeout: float) -> None:
        budget = min(timeout, left())
        if budget < 30.0:
            main_line[key] = {"error": f"child skipped: {max(budget, 0.0):.0f} s left of the "
                                       f"{args.deadline:.0f} s deadline"}
            return
        # the extra configs time at most --extra-steps whole waves (after at most 2 warm-up waves):
        # enough for a stable number, and the 70B / Mixtral children then fit the one deadline
        steps = ["--steps", str(min(args.steps, args.extra_steps)), "--warmup", str(min(args.warmup, 2))]
        trc, tl, wall = run_child(_strip(argv, strip) + cargs + steps + ["--tp-extra-model", "none",
                                                                         "--ep-extra-model", "none", "--child"],
                                  args.gpus, budget)
        if tl is not None:
            main_line[key] = {k: tl.get(k) for k in ("value", "unit", "p50_e2e_latency_ms", "ms_per_step", "steps",
                                                     "warmup", "scaling")}
            main_line[key].update(model=tl["config"]["model"], parallelism=tl["config"]["parallelism"],
                                  rpc=tl["config"].get("rpc"),
                                  global_batch=tl["config"]["global_batch"], init_s=tl["config"].get("init_s"),
                                  wall_s=round(wall, 1))
        else:
            main_line[key] = {"error": f"child rc {trc}" + (f" (timeout after {budget:.0f} s)" if trc == 124 else ""),
                              "wall_s": round(wall, 1)}

    if args.tp == 1 and args.ep == 1:
        extra = args.tp_extra_model
        if extra == "auto":
            extra = "llama3-70b" if args.model == "llama3-8b" else "none"
        if extra and extra != "none":
            extra_child(_extra_key("tp", args.gpus, extra), ["--model", extra, "--tp", str(args.gpus), "--mode",
                                                             args.tp_extra_mode], args.tp_extra_timeout)
        moe = args.ep_extra_model
        if moe == "auto":
            moe = "mixtral-8x7b" if args.model == "llama3-8b" and 8 % args.gpus == 0 else "none"
        if moe and moe != "none":
            extra_child(_extra_key("ep", args.gpus, moe), ["--model", moe, "--tp", "1", "--ep", str(args.gpus),
                                                           "--mode", args.mode], args.ep_extra_timeout)
    print(json.dumps(main_line), flush=True)
    return 0


async def _abarrier(group) -> None:
    """A barrier that keeps this rank's event loop (and its gRPC server) running."""
    import torch.distributed as dist
    await asyncio.get_running_loop().run_in_executor(None, lambda: dist.barrier(group=group))


async def run_waves(args, engine, st, leaders_group, llm=None, n_replicas=1):
    import grpc
    import torch
    import torch.distributed as dist

    from polykey_service_amd import proto
    from polykey_service_amd.adapters.local_llm import attach_local_llm
    from polykey_service_amd.config.server_config import ServerConfig
    from polykey_service_amd.server import PolykeyServer
    from polykey_service_amd.service import ToolRouter
    from polykey_service_amd.utils import slog

    logger = slog.Logger(open(os.devnull, "w"))
    router = ToolRouter()
    cfg = ServerConfig(model=args.model, backend="local")
    attach_local_llm(router, cfg, logger, engine=engine, llm=llm)
    conc = args.concurrency * n_replicas  # single front end: every replica's clients
    port = args.port_base + st.rank if args.port_base > 0 else 0
    srv = PolykeyServer(router, logger, f"127.0.0.1:{port}")
    port = await srv.start()
    if args.client == "process":
        try:
            return await _drive_external(args, engine, st, leaders_group if n_replicas == 1 else None, port, srv,
                                         llm=router.llm, conc=args.concurrency * n_replicas,
                                         stop_after=engine.lockstep or n_replicas > 1)
        finally:
            await srv.server.stop(0)
    http = session = None
    if args.mode == "openai":
        # the OpenAI-compatible route on the same process and event loop as the gRPC server
        import aiohttp

        from polykey_service_amd.api.openai import serve_openai
        hport = _free_port()
        http = await serve_openai(router, f"127.0.0.1:{hport}", logger)
        session = aiohttp.ClientSession(connector=aiohttp.TCPConnector(limit=0),
                                        timeout=aiohttp.ClientTimeout(total=600))
        url = f"http://127.0.0.1:{hport}/v1/chat/completions"
        for _ in range(600):  # the route is up once it answers
            try:
                async with session.get(f"http://127.0.0.1:{hport}/health") as hr:
                    if hr.status == 200:
                        break
            except aiohttp.ClientError:
                pass
            await asyncio.sleep(0.05)
        tok = router.llm.tokenizer
        # prompt length in tokens after the chat template: the content is sized so the templated
        # prompt is exactly --prompt-len tokens (byte tokenizer: one ASCII character per token)
        overhead = len(tok.encode(tok.apply_chat_template([{"role": "user", "content": ""}])))
        if args.prompt_len <= overhead:
            raise SystemExit(f"--prompt-len {args.prompt_len}: the chat template alone is {overhead} tokens")
    channel = grpc.aio.insecure_channel(f"127.0.0.1:{port}", options=[
        ("grpc.max_receive_message_length", 64 << 20), ("grpc.max_send_message_length", 64 << 20)])
    unary = channel.unary_unary(proto.EXECUTE_TOOL, request_serializer=proto.ExecuteToolRequest.SerializeToString,
                                response_deserializer=proto.ExecuteToolResponse.FromString)
    stream = channel.unary_stream(proto.EXECUTE_TOOL_STREAM,
                                  request_serializer=proto.ExecuteToolRequest.SerializeToString,
                                  response_deserializer=proto.ExecuteToolResponse.FromString)
    V = engine.mcfg.vocab_size
    rng = random.Random(args.seed * 1000 + st.rank)
    tool = f"llm.generate:{args.model}"
    llm = router.llm
    # single front end: the other ranks sit in their engine servers, so rank 0 times the waves alone
    sync_ranks = dist.is_initialized() and n_replicas == 1

    timing = os.environ.get("POLYKEY_BENCH_TIMING") == "1"
    marks = []

    def build():
        if args.mode == "openai":
            n = max(1, args.prompt_len - overhead)
            text = "".join(rng.choice("abcdefghijklmnopqrstuvwxyz ") for _ in range(n))
            return {"messages": [{"role": "user", "content": text}], "max_tokens": args.max_tokens,
                    "ignore_eos": True, "temperature": 0.0}
        req = proto.ExecuteToolRequest(tool_name=tool)
        req.parameters.update({"prompt_token_ids": [rng.randrange(0, V) for _ in range(args.prompt_len)],
                               "max_tokens": args.max_tokens, "ignore_eos": True, "temperature": 0.0,
                               "return": "struct"})
        return req

    async def one(req):
        t0 = time.perf_counter()  # submit time (requests are prebuilt: see `waves` below)
        if args.mode == "openai":
            async with session.post(url, json=req) as hr:
                body = await hr.json()
            if hr.status != 200:
                raise RuntimeError(f"openai route: HTTP {hr.status}: {body}")
            return int(body["usage"]["completion_tokens"]), time.perf_counter() - t0
        if args.mode == "unary":
            resp = await unary(req, timeout=600)
        else:
            resp = None
            async for resp in stream(req, timeout=600):
                pass
        t1 = time.perf_counter()
        dt = t1 - t0
        usage = resp.struct_output.fields["usage"].struct_value.fields
        if timing:
            m = proto.struct_to_dict(resp.struct_output)["metrics"]
            marks.append((t0, t1, m))
        return int(usage["completion_tokens"].number_value), dt

    async def wave(reqs):
        marks.clear()
        tw = time.perf_counter()
        res = await asyncio.gather(*[one(r) for r in reqs])
        if timing and marks:
            # host-side breakdown of the wave (stderr): request build/submit span, the engine's
            # view (queue, TTFT, e2e) and what the RPC path adds on top of it
            te = time.perf_counter()
            sub = max(m[0] for m in marks) - tw
            rpc = sorted((m[1] - m[0]) - m[2]["server_e2e_s"] for m in marks)
            # the two legs (in-process clients share the server's monotonic clock)
            rin = sorted(m[2]["server_t0"] - m[0] for m in marks if "server_t0" in m[2]) or [0.0]
            rout = sorted(m[1] - m[2]["server_t0"] - m[2]["server_e2e_s"] for m in marks if "server_t0" in m[2]) or [0.0]
            ttft = sorted(m[2].get("ttft_s", 0.0) for m in marks)
            e2e = sorted(m[2].get("e2e_s", 0.0) for m in marks)
            print(f"[wave] wall {1e3 * (te - tw):.1f} ms | last submit +{1e3 * sub:.1f} ms | engine e2e "
                  f"min/max {1e3 * e2e[0]:.1f}/{1e3 * e2e[-1]:.1f} ms | ttft min/max {1e3 * ttft[0]:.1f}/"
                  f"{1e3 * ttft[-1]:.1f} ms | rpc overhead p50/max {1e3 * rpc[len(rpc) // 2]:.2f}/{1e3 * rpc[-1]:.2f} ms "
                  f"(request leg {1e3 * rin[len(rin) // 2]:.2f}/{1e3 * rin[-1]:.2f}, response leg "
                  f"{1e3 * rout[len(rout) // 2]:.2f}/{1e3 * rout[-1]:.2f}) | "
                  f"last response +{1e3 * (max(m[1] for m in marks) - tw):.1f} ms", file=sys.stderr, flush=True)
        return sum(r[0] for r in res), [r[1] for r in res]

    for _ in range(args.warmup):
        await wave([build() for _ in range(conc)])
    # the load generator prepares its synthetic requests up front, as a separate client
    # process would: building 64 x 256 random ids inside a wave would only steal the event
    # loop (and the GIL) from the server under test
    waves = [[build() for _ in range(conc)] for _ in range(args.steps)]
    dev = engine.device
    if sync_ranks:
        await _abarrier(leaders_group)
    if dev.type == "cuda":
        torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    tokens, lats = 0, []
    for reqs in waves:
        n, l = await wave(reqs)
        tokens += n
        lats += l
    if dev.type == "cuda":
        torch.cuda.synchronize(dev)
    if sync_ranks:
        await _abarrier(leaders_group)
    elapsed = time.perf_counter() - t0
    await channel.close()
    if session is not None:
        await session.close()
        await http.shutdown()
    await srv.server.stop(0)
    if engine.lockstep or n_replicas > 1:
        # DP attention + EP: leave the lockstep loop together with the other ranks; single front
        # end: stop the other ranks' engine servers (they are waiting on it)
        await asyncio.get_running_loop().run_in_executor(None, llm.shutdown)
    return tokens, elapsed, lats


async def _drive_external(args, engine, st, leaders_group, port, srv, llm, conc, stop_after):
    """Waves from a load-generator child process (no exec: a fresh interpreter via
    create_subprocess_exec); the timed span is bracketed here by barrier + device sync."""
    import torch
    import torch.distributed as dist
    cmd = [sys.executable, "-m", "polykey_service_amd.client.load_gen", "--addr", f"127.0.0.1:{port}",
           "--tool", f"llm.generate:{args.model}", "--vocab", str(engine.mcfg.vocab_size),
           "--concurrency", str(conc), "--prompt-len", str(args.prompt_len),
           "--max-tokens", str(args.max_tokens), "--mode", args.mode, "--steps", str(args.steps),
           "--warmup", str(args.warmup), "--seed", str(args.seed * 1000 + st.rank)]
    env = dict(os.environ, PYTHONPATH=os.path.dirname(os.path.abspath(__file__)) + os.pathsep
               + os.environ.get("PYTHONPATH", ""))
    proc = await asyncio.create_subprocess_exec(*cmd, stdin=asyncio.subprocess.PIPE,
                                                stdout=asyncio.subprocess.PIPE, env=env)
    try:
        ready = json.loads((await proc.stdout.readline()) or b"{}")
        if not ready.get("ready"):
            raise RuntimeError(f"load generator failed to start: {ready}")
        dev = engine.device
        if dist.is_initialized() and leaders_group is not None:
            await _abarrier(leaders_group)
        if dev.type == "cuda":
            torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        proc.stdin.write(b"go\n")
        await proc.stdin.drain()
        res = json.loads((await proc.stdout.readline()) or b"{}")
        if dev.type == "cuda":
            torch.cuda.synchronize(dev)
        if dist.is_initialized() and leaders_group is not None:
            await _abarrier(leaders_group)
        elapsed = time.perf_counter() - t0
        if "tokens" not in res:
            raise RuntimeError(f"load generator failed: {res}")
    finally:
        if proc.returncode is None:
            try:
                proc.stdin.close()  # a generator still waiting for "go" reads EOF and exits
            except Exception:
                pass
            try:
                await asyncio.wait_for(proc.wait(), 30)
            except asyncio.TimeoutError:
                proc.kill()
    if stop_after:  # DP attention + EP lockstep / single-front-end engine servers: stop with the other ranks
        await asyncio.get_running_loop().run_in_executor(None, llm.shutdown)
    return res["tokens"], elapsed, res["lats"]


def main(argv=None) -> int:
    argv = list(sys.argv[1:] if argv is None else argv)
    args = parse_args(argv)
    if args.gpus > 1 and not args.child:
        if int(os.environ.get("RANK", "0")) != 0:
            return 0  # under the driver's torchrun: rank 0 runs the measurement children
        return orchestrate(args, argv)
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    import torch
    import torch.distributed as dist

    from polykey_service_amd.engine.llm_engine import EngineConfig, LLMEngine
    from polykey_service_amd.parallel.state import init_parallel

    st = init_parallel(tp=args.tp, ep=args.ep)
    max_len = args.prompt_len + args.max_tokens + 32
    max_len = (max_len + 511) // 512 * 512
    seqs = max(args.concurrency, 1)
    if args.frontend != "replicas" and st.world_size > 1 and st.tp_size == 1 and not st.dp_attention:
        # a routed front end balances only approximately: an engine that gets a few requests more
        # than its share must still batch them all (a request over max_num_seqs would wait a
        # whole wave) -- headroom up to the next graph bucket
        seqs = seqs * 3 // 2
    ecfg = EngineConfig(model=args.model, seed=args.seed, max_num_seqs=seqs,
                        max_num_batched_tokens=args.max_batched_tokens, max_model_len=max_len,
                        hip_graphs=not args.no_graphs, num_kv_blocks=args.num_kv_blocks,
                        gpu_mem_fraction=args.gpu_mem_fraction)
    if args.mode == "openai":
        # every templated chat prompt starts with the same markup: the prefix cache would serve
        # those blocks and skip their prefill work -- off, so no work is skipped in the timed region
        ecfg.prefix_caching = False
    t_init = time.perf_counter()
    engine = LLMEngine(ecfg, st)
    if engine.device.type == "cuda":
        torch.cuda.synchronize(engine.device)  # weight init / packing / graph capture run asynchronously
    if dist.is_initialized():
        dist.barrier()
    init_s = time.perf_counter() - t_init
    from polykey_service_amd.utils import test_hooks
    if test_hooks.get("POLYKEY_BENCH_HANG") == "tp" and st.tp_size > 1:
        while True:  # a hung TP child (tests: the orchestrator's deadline must still print the line)
            time.sleep(60)
    leaders = list(range(0, st.world_size, st.tp_size))
    leaders_group = dist.new_group(leaders) if dist.is_initialized() else None
    dp_front = st.world_size > 1 and st.tp_size == 1 and not engine.lockstep
    if args.frontend == "single" and dp_front:
        from polykey_service_amd.engine.async_llm import AsyncLLM
        from polykey_service_amd.engine.remote import dp_gateway
        local = AsyncLLM(engine)
        pool = dp_gateway(local, st)  # ranks > 0 serve their engine until rank 0 stops them
        if pool is None:
            local.shutdown()
            tokens, elapsed, lats = 0, 0.0, []
        else:
            tokens, elapsed, lats = asyncio.run(run_waves(args, engine, st, None, llm=pool, n_replicas=st.world_size))
    elif st.tp_rank != 0:
        engine.runner.worker_loop()
        tokens, elapsed, lats = 0, 0.0, []
    else:
        tokens, elapsed, lats = asyncio.run(run_waves(args, engine, st, leaders_group))
        engine.runner.stop_workers()

    if dist.is_initialized():
        # TP workers contribute (0 tokens, 0 s, no latencies); elapsed = max over ranks
        allr = [None] * st.world_size
        dist.all_gather_object(allr, (tokens, elapsed, lats, engine.scheduler.num_cached_tokens))
        tokens = sum(x[0] for x in allr)
        elapsed = max(x[1] for x in allr)
        lats = [l for x in allr for l in x[2]]
        cached = sum(x[3] for x in allr)
    else:
        cached = engine.scheduler.num_cached_tokens
    if st.rank == 0:
        p50 = statistics.median(lats) if lats else None
        value = tokens / elapsed if elapsed > 0 else 0.0
        out = {
            "metric": METRIC,
            "value": round(value, 2),
            "unit": "output_tokens/s",
            "n_gpus": st.world_size,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / max(args.steps, 1) * 1000.0, 3),
            "higher_is_better": True,
            "scaling": "strong" if st.tp_size > 1 and st.dp_size == 1 else "weak",
            "vs_baseline": None,
            "dtype": "bf16",
            "data": "synthetic (random prompt token ids, random-init weights, ignore_eos)",
            "p50_e2e_latency_ms": round(p50 * 1000.0, 2) if p50 else None,
            "config": {
                "model": MODEL_NAMES.get(args.model, args.model),
                "global_batch": args.concurrency * (st.world_size // st.tp_size),
                "seq_len": args.prompt_len,
                "output_len": args.max_tokens,
                "parallelism": (f"tp{st.tp_size}" + (f"_dp{st.dp_size}" if st.dp_size > 1 else "")
                                + (f"_ep{st.ep_size}" if st.ep_size > 1 else "")) if st.tp_size > 1
                else f"dp{st.world_size}" + (f"_ep{st.ep_size}_a2a" if st.ep_size > 1 else "")
                + ("_single_frontend" if args.frontend == "single" and dp_front else ""),
                "concurrency_per_replica": args.concurrency,
                "rpc": "POST /v1/chat/completions (OpenAI route)" if args.mode == "openai" else
                f"ExecuteTool ({args.mode})",
                "clients": "load-generator process" if args.client == "process" else "server event loop",
                "hip_graphs": not args.no_graphs,
                # every prompt is unique, so the prefix cache must serve nothing (no skipped work)
                "prefix_caching": ecfg.prefix_caching,
                "prefix_cache_hit_tokens": cached,
                "init_s": round(init_s, 1),
            },
        }
        print(json.dumps(out), flush=True)
    if dist.is_initialized():
        dist.barrier()
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
