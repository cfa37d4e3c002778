"""On-node LLM adapter: the replacement for the reference's (absent) third-party HTTP
provider layer (``internal/adapters``).

Registers model tools on the :class:`ToolRouter`:

* ``llm.generate:<model>`` — ``parameters = {prompt | prompt_token_ids, max_tokens, temperature,
  top_p, top_k, min_p, seed, ignore_eos, stop, stop_token_ids, return: "text"|"struct"}``
* ``llm.chat:<model>``     — same with ``messages = [{role, content}, ...]``, and optionally
  OpenAI ``tools`` / ``tool_choice`` plus ``execute_tools`` / ``tool_secret_id`` /
  ``max_tool_rounds`` (service/tool_calls.py): the struct output then also carries
  ``tool_calls`` and ``tool_results``

Unary ``ExecuteTool`` returns the completion as ``string_output`` (what the reference's dev
client logs), or a ``struct_output`` ``{text, finish_reason, usage, metrics}`` when
``return == "struct"``.  ``ExecuteToolStream`` yields ``string_output`` deltas (tokens that
arrived together are coalesced into one message) and ends with the struct summary.
"""
from __future__ import annotations

import time
from typing import Dict, List, Optional

from .. import proto
from ..engine.sequence import SamplingParams
from ..engine.tokenizer import IncrementalDetokenizer
from ..service.base import RequestContext, ToolError, ok_status
from ..service.tool_calls import run_chat, tool_rounds, validate_tools


def _status():
    return ok_status()


class LLMTool:
    requires_secret = False

    def __init__(self, name: str, model_name: str, llm, chat: bool):
        self.name = name
        self.model_name = model_name
        self.llm = llm
        self.chat = chat
        self.tok = llm.tokenizer
        self.router = None  # set by attach_local_llm: executes model-emitted tool calls

    # ------------------------------------------------------------- params
    def _prompt(self, params: dict) -> List[int]:
        if "prompt_token_ids" in params:
            return [int(x) for x in params["prompt_token_ids"]]
        if self.chat:
            msgs = params.get("messages")
            if not isinstance(msgs, list) or not msgs:
                raise ToolError("INVALID_ARGUMENT", "llm.chat requires a non-empty 'messages' list")
            text = self.tok.apply_chat_template(msgs)
        else:
            text = params.get("prompt")
            if not isinstance(text, str) or not text:
                raise ToolError("INVALID_ARGUMENT", "llm.generate requires 'prompt' (string) or 'prompt_token_ids'")
        return self.tok.encode(text)

    def _sampling(self, params: dict) -> SamplingParams:
        try:
            sp = SamplingParams.from_dict(params)
            sp.validate(1 << 30)
        except (ValueError, TypeError) as e:
            raise ToolError("INVALID_ARGUMENT", str(e))
        return sp

    def _summary(self, text: str, n_prompt: int, toks: List[int], last, t0: float, with_ids: bool = False) -> dict:
        m = (last.metrics or {}) if last is not None else {}
        out = {
            "model": self.model_name,
            "text": text,
            "finish_reason": last.finish_reason if last is not None else "abort",
            "usage": {"prompt_tokens": n_prompt, "completion_tokens": len(toks),
                      "total_tokens": n_prompt + len(toks)},
            # server_t0: the handler's start on the monotonic clock (an in-process client can split
            # its round trip into the request and response legs)
            "metrics": {k: v for k, v in {**m, "server_e2e_s": time.monotonic() - t0, "server_t0": t0}.items()
                        if v is not None},
        }
        if with_ids:  # parameters.return_token_ids: the generated ids themselves (token-level clients, tests)
            out["token_ids"] = list(toks)
        return out

    @staticmethod
    def _stop_hit(text: str, stops) -> Optional[int]:
        for s in stops or ():
            i = text.find(s)
            if i >= 0:
                return i
        return None

    def _tools(self, params: dict):
        """(tools, tool_choice) when this chat request uses function tools, else None."""
        if not self.chat or not (params.get("tools") or params.get("tool_choice")):
            return None
        try:
            tools, choice = validate_tools(params.get("tools"), params.get("tool_choice"))
        except ValueError as e:
            raise ToolError("INVALID_ARGUMENT", str(e))
        return (tools, choice) if tools and choice != "none" else None

    async def _run_tools(self, ctx: RequestContext, params: dict, tc) -> "proto.ExecuteToolResponse":
        t0 = time.monotonic()
        msgs = params.get("messages")
        if not isinstance(msgs, list) or not msgs:
            raise ToolError("INVALID_ARGUMENT", "llm.chat requires a non-empty 'messages' list")
        sp = self._sampling(params)
        try:
            rounds = tool_rounds(params.get("max_tool_rounds"))
        except ValueError as e:
            raise ToolError("INVALID_ARGUMENT", str(e))
        oc = await run_chat(self.llm, self.tok.chat_template, msgs, sp, tc[0], tc[1], router=self.router,
                            execute=bool(params.get("execute_tools")), secret_id=params.get("tool_secret_id"),
                            max_rounds=rounds, request_id=ctx.request_id)
        resp = proto.ExecuteToolResponse(status=_status())
        if params.get("return") == "struct" or oc.tool_calls or oc.executed:
            m = oc.metrics or {}
            resp.struct_output.update({
                "model": self.model_name, "text": oc.content, "tool_calls": oc.tool_calls,
                "tool_results": oc.executed, "finish_reason": oc.finish_reason,
                "usage": {"prompt_tokens": oc.prompt_tokens, "completion_tokens": oc.completion_tokens,
                          "total_tokens": oc.prompt_tokens + oc.completion_tokens},
                "metrics": {k: v for k, v in {**m, "server_e2e_s": time.monotonic() - t0}.items() if v is not None}})
        else:
            resp.string_output = oc.content
        return resp

    # ------------------------------------------------------------- tool API
    async def run(self, ctx: RequestContext, params: dict, secret, metadata: Dict[str, str]):
        tc = self._tools(params)
        if tc is not None:
            return await self._run_tools(ctx, params, tc)
        t0 = time.monotonic()
        prompt = self._prompt(params)
        sp = self._sampling(params)
        toks: List[int] = []
        last = None
        text = ""
        # without stop strings a unary call needs only the final result: a remote engine
        # (engine/remote.py) then reports the request once instead of once per step
        async for out in self.llm.generate(prompt, sp, request_id=ctx.request_id, final_only=not sp.stop):
            toks.extend(out.new_token_ids)
            last = out
            if sp.stop:
                text = self.tok.decode(toks)
                cut = self._stop_hit(text, sp.stop)
                if cut is not None:
                    text = text[:cut]
                    break
        if not sp.stop:
            text = self.tok.decode(toks)
        resp = proto.ExecuteToolResponse(status=_status())
        if params.get("return") == "struct":
            resp.struct_output.update(self._summary(text, len(prompt), toks, last, t0, bool(params.get("return_token_ids"))))
        else:
            resp.string_output = text
        return resp

    async def stream(self, ctx: RequestContext, params: dict, secret, metadata: Dict[str, str]):
        tc = self._tools(params)
        if tc is not None:  # a tool-enabled chat is decided whole: one final message
            yield await self._run_tools(ctx, params, tc)
            return
        t0 = time.monotonic()
        prompt = self._prompt(params)
        sp = self._sampling(params)
        toks: List[int] = []
        last = None
        detok = IncrementalDetokenizer(self.tok)
        agen = self.llm.generate(prompt, sp, request_id=ctx.request_id)
        try:
            async for out in agen:
                toks.extend(out.new_token_ids)
                last = out
                before = len(detok.text)
                delta = detok.push(out.new_token_ids)
                cut = self._stop_hit(detok.text, sp.stop) if sp.stop else None
                if cut is not None:
                    delta = detok.text[before:cut] if cut > before else ""
                    detok.text = detok.text[:cut]
                if delta:
                    yield proto.ExecuteToolResponse(string_output=delta)
                if cut is not None:
                    break
            else:
                tail = detok.flush()
                if tail:
                    yield proto.ExecuteToolResponse(string_output=tail)
        finally:
            await agen.aclose()
        text = detok.text
        final = proto.ExecuteToolResponse(status=_status())
        final.struct_output.update(self._summary(text, len(prompt), toks, last, t0, bool(params.get("return_token_ids"))))
        yield final


class ReplicaPool:
    """Request-level data parallelism behind one front end (SURVEY.md §2.3 "DP"): every
    request goes to the replica with the fewest unfinished requests.  Replicas are in-process
    :class:`AsyncLLM` engines (one thread and HIP device each) or
    :class:`~polykey_service_amd.engine.remote.RemoteEngine` handles of engine processes (one
    rank per GPU: :func:`~polykey_service_amd.engine.remote.dp_gateway`, or the TP groups of
    :func:`attach_model_groups`).  Duck-types :class:`AsyncLLM`."""

    def __init__(self, replicas):
        self.replicas = list(replicas)
        self.tokenizer = self.replicas[0].tokenizer
        self.engine = getattr(self.replicas[0], "engine", None)  # None: every replica is remote
        self.on_fatal = None
        self.watchdog_s = 0.0

    def _pick(self):
        return min(self.replicas, key=lambda r: r.load())

    def load(self) -> int:
        return sum(r.load() for r in self.replicas)

    def generate(self, prompt_ids, params, request_id=None, final_only=False):
        return self._pick().generate(prompt_ids, params, request_id, final_only=final_only)

    async def generate_all(self, prompt_ids, params, request_id=None):
        return await self._pick().generate_all(prompt_ids, params, request_id)

    def healthy(self) -> bool:
        return all(r.healthy() for r in self.replicas)

    def __setattr__(self, k, v):
        object.__setattr__(self, k, v)
        if k in ("on_fatal", "watchdog_s") and "replicas" in self.__dict__:
            for r in self.replicas:
                setattr(r, k, v)

    def shutdown(self, timeout: float = 10.0) -> None:
        # remote handles first: their "stop" frames release the other ranks' engine servers
        local = [r for r in self.replicas if hasattr(r, "engine")]
        for r in self.replicas:
            if r not in local:
                r.shutdown(timeout)
        for r in local:
            r.shutdown(timeout)

    async def aclose(self) -> None:
        for r in self.replicas:
            await r.aclose()


class ModelSet:
    """Several served models behind one front end (``ServerConfig.serve_models``): duck-types the
    backend face the server watches -- healthy only while every model's engines are, one fatal
    handler and watchdog for all of them, closed together."""

    def __init__(self, llms: Dict[str, object]):
        self.llms = dict(llms)
        self.on_fatal = None
        self.watchdog_s = 0.0

    def __setattr__(self, k, v):
        object.__setattr__(self, k, v)
        if k in ("on_fatal", "watchdog_s") and "llms" in self.__dict__:
            for llm in self.llms.values():
                setattr(llm, k, v)

    def healthy(self) -> bool:
        return all(llm.healthy() for llm in self.llms.values())

    def load(self) -> int:
        return sum(llm.load() for llm in self.llms.values())

    def shutdown(self, timeout: float = 10.0) -> None:
        for llm in self.llms.values():
            llm.shutdown(timeout)

    async def aclose(self) -> None:
        for llm in self.llms.values():
            await llm.aclose()


def parse_serve_models(spec: str) -> List[tuple]:
    """``"llama3-8b@0-3,mixtral-8x7b@4,tiny"`` -> [("llama3-8b", [0, 1, 2, 3]), ("mixtral-8x7b", [4]),
    ("tiny", [])] (no ``@``: the next free device).  Entries of one process: TP = 1 only (a
    ``:tp<N>`` entry needs one process per GPU: :func:`plan_model_groups`)."""
    out = []
    for name, devs, tp in parse_serve_plan(spec):
        if tp != 1:
            raise ValueError(f"serve_models entry {name!r} asks for tp={tp}: tensor parallel models are served by "
                             "one process per GPU (torchrun), not by a single process")
        out.append((name, devs))
    return out


def parse_serve_plan(spec: str) -> List[tuple]:
    """``"llama3-70b@0-3:tp4,llama3-8b@4,mixtral-8x7b@5-6"`` -> [("llama3-70b", [0..3], 4),
    ("llama3-8b", [4], 1), ("mixtral-8x7b", [5, 6], 1)]: model, devices (no ``@``: the next free
    ones) and its TP degree (``:tp<N>``, default 1; the devices form len(devices) / N replicas)."""
    out = []
    for item in (x.strip() for x in spec.split(",")):
        if not item:
            continue
        item, _, tps = item.partition(":")
        tp = 1
        if tps:
            if not tps.startswith("tp") or not tps[2:].isdigit() or int(tps[2:]) < 1:
                raise ValueError(f"serve_models entry {item!r}: bad TP suffix {tps!r} (':tp<N>')")
            tp = int(tps[2:])
        name, _, dev = item.partition("@")
        if not name:
            raise ValueError(f"serve_models entry {item!r} has no model name")
        if not dev:
            devs: List[int] = []
        elif "-" in dev:
            a, b = (int(v) for v in dev.split("-"))
            if b < a:
                raise ValueError(f"serve_models entry {item!r}: empty device range")
            devs = list(range(a, b + 1))
        else:
            devs = [int(dev)]
        if devs and len(devs) % tp:
            raise ValueError(f"serve_models entry {item!r}: {len(devs)} devices are not a multiple of tp={tp}")
        out.append((name, devs, tp))
    names = [n for n, _, _ in out]
    if len(set(names)) != len(names):
        raise ValueError(f"serve_models names a model twice: {spec!r}")
    return out


def plan_model_groups(spec: str, world: int) -> List[tuple]:
    """The TP groups of a one-process-per-GPU job serving ``spec`` on ``world`` ranks (rank r on GPU
    r): [(model, [ranks]), ...], each group TP over consecutive ranks, the lowest its leader.  An
    entry without ``@`` takes the next free ranks (tp of them); every rank must serve exactly one
    group, and rank 0 -- the front end -- leads the first group it is in."""
    entries = parse_serve_plan(spec)
    taken = sorted(d for _, devs, _ in entries for d in devs)
    if len(set(taken)) != len(taken):
        raise ValueError(f"serve_models gives a GPU to two models: {spec!r}")
    free = [r for r in range(world) if r not in taken]
    groups = []
    for name, devs, tp in entries:
        if not devs:
            if len(free) < tp:
                raise ValueError(f"model {name!r} needs {tp} more GPU(s); the job has {world} ranks ({spec!r})")
            devs, free = free[:tp], free[tp:]
        for i in range(0, len(devs), tp):
            g = devs[i:i + tp]
            if g != list(range(g[0], g[0] + tp)):
                raise ValueError(f"model {name!r}: a TP group must be consecutive GPUs, got {g}")
            groups.append((name, g))
    used = sorted(r for _, g in groups for r in g)
    if used != list(range(world)):
        raise ValueError(f"serve_models {spec!r} covers ranks {used}, the job has {world} (one per GPU, each "
                         "serving exactly one model)")
    return groups


def attach_models(router, cfg, logger) -> ModelSet:
    """Build every model of ``cfg.serve_models`` (one process; each model's engines on their own
    devices, one engine thread each) and register its tools; the first listed is the default for
    ``llm.chat`` / ``llm.generate`` without a model."""
    import dataclasses as _dc

    import torch

    from ..engine.async_llm import AsyncLLM, device_guard
    from ..engine.llm_engine import EngineConfig, LLMEngine
    from ..parallel.state import ParallelState
    entries = parse_serve_models(cfg.serve_models)
    n_dev = torch.cuda.device_count() if torch.cuda.is_available() and cfg.device != "cpu" else 0
    taken = {d for _, devs in entries for d in devs}
    free = iter([d for d in range(max(n_dev, 1)) if d not in taken])
    llms = {}
    for name, devs in entries:
        if not devs:
            d = next(free, None)
            if d is None and n_dev:
                raise ValueError(f"model {name!r} has no device left: every GPU of this node is taken "
                                 f"({cfg.serve_models!r}); give it one with '@<gpu>'")
            devs = [d or 0]
        engines = []
        for d in devs:
            if n_dev and d >= n_dev:
                raise ValueError(f"model {name!r} asks for GPU {d}; this node has {n_dev}")
            dev = torch.device(f"cuda:{d}") if n_dev else torch.device("cpu")
            ecfg = _dc.replace(EngineConfig.from_server_config(_dc.replace(cfg, model=name)), device=str(dev))
            # the engine's weights, KV cache and warm-up launches on ITS device (the native ops
            # launch on the thread's current device); its AsyncLLM thread binds the same device
            with device_guard(dev):
                engines.append(LLMEngine(ecfg, ParallelState(device=dev)))
        llm = AsyncLLM(engines[0]) if len(engines) == 1 else ReplicaPool([AsyncLLM(e) for e in engines])
        attach_local_llm(router, _dc.replace(cfg, model=name), logger, engine=engines[0], llm=llm)
        llms[name] = llm
    router.llm = ModelSet(llms)
    return router.llm


def attach_model_groups(router, cfg, logger, timeout_s: float = 600.0) -> Optional[ModelSet]:
    """Several models behind ONE front end on a one-process-per-GPU job (torchrun), each model
    served by TP groups of its own (``serve_models`` entries ``name@<gpus>[:tp<N>]``, e.g.
    ``llama3-70b@0-3:tp4,llama3-8b@4,mixtral-8x7b@5-6``): the world is split into the groups of
    :func:`plan_model_groups`, every rank builds its group's engine, each group's leader serves its
    engine to rank 0 over the engine wire (engine/remote.py), the other ranks of a group follow
    their leader's steps (TP workers), and rank 0 registers ``llm.*:<model>`` for every model,
    routed least-loaded over that model's groups.  Rank 0 returns the :class:`ModelSet`; the other
    ranks return None once the front end has stopped them (the caller exits)."""
    import dataclasses as _dc
    import os
    import secrets
    import socket as _socket

    import torch.distributed as dist

    from ..engine.async_llm import AsyncLLM
    from ..engine.llm_engine import EngineConfig, LLMEngine, tokenizer_for
    from ..engine.remote import EngineServer, RemoteEngine
    from ..parallel.state import init_parallel

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    groups = plan_model_groups(cfg.serve_models, world)
    name = next(n for n, g in groups if rank in g)
    st = init_parallel(tp_groups=[g for _, g in groups], timeout_s=timeout_s,
                       device=None if cfg.device in ("", "cuda") else cfg.device)
    ecfg = EngineConfig.from_server_config(_dc.replace(cfg, model=name))
    engine = LLMEngine(ecfg, st)
    # the leaders' engine-server addresses, exchanged before the workers enter their step loops
    single_node = int(os.environ.get("LOCAL_WORLD_SIZE", str(world))) == world
    bind = "127.0.0.1" if single_node else "0.0.0.0"
    advertise = os.environ.get("POLYKEY_GATEWAY_HOST") or ("127.0.0.1" if single_node else _socket.gethostname())
    tok = [secrets.token_hex(16) if rank == 0 else None]
    dist.broadcast_object_list(tok, src=0, group=st.world_cpu_group)
    llm = AsyncLLM(engine) if st.tp_rank == 0 else None
    server = EngineServer(llm, host=bind, token=tok[0]) if llm is not None and rank != 0 else None
    addrs: List = [None] * world
    dist.all_gather_object(addrs, (advertise, server.port) if server is not None else None, group=st.world_cpu_group)
    if st.tp_rank != 0:
        try:
            engine.runner.worker_loop()  # until the group's leader stops it
        except BaseException as e:  # noqa: BLE001 - leader died / collective failed
            logger.error("TP worker failed", error=repr(e), rank=rank, model=name)
            raise
        return None
    if server is not None:
        logger.info("model group leader serving", model=name, rank=rank, tp=st.tp_size, port=server.port)
        try:
            server.serve()  # until the front end stops it
        finally:
            llm.shutdown()  # (stops the group's TP workers too)
        return None
    # rank 0: the front end
    llms: Dict[str, object] = {}
    for mname in dict.fromkeys(n for n, _ in groups):
        tk = tokenizer_for(_dc.replace(ecfg, model=mname))
        reps = []
        for n, g in groups:
            if n != mname:
                continue
            reps.append(llm if g[0] == 0 else RemoteEngine(tuple(addrs[g[0]]), tk, name=f"{n}@rank{g[0]}",
                                                         token=tok[0]))
        pool = reps[0] if len(reps) == 1 else ReplicaPool(reps)
        mcfg = _dc.replace(cfg, model=mname)
        _register_tools(router, mcfg, pool)
        llms[mname] = pool
        logger.info("model group ready", model=mname, groups=[g for n, g in groups if n == mname])
    router.llm = ModelSet(llms)
    return router.llm


def _register_tools(router, cfg, llm) -> None:
    name = cfg.model if isinstance(cfg.model, str) else "model"
    router.register_model_tool("llm.generate", name, LLMTool("llm.generate", name, llm, chat=False))
    chat_tool = LLMTool("llm.chat", name, llm, chat=True)
    chat_tool.router = router
    router.register_model_tool("llm.chat", name, chat_tool)


def attach_local_llm(router, cfg, logger, engine=None, llm=None):
    """Build (or reuse) the engine for ``cfg.model`` and register its tools (``llm``: an already
    built AsyncLLM / ReplicaPool over ``engine``)."""
    from ..engine.async_llm import AsyncLLM
    from ..engine.llm_engine import EngineConfig, LLMEngine
    from ..parallel.state import init_parallel

    if llm is not None:
        pass
    elif engine is None and getattr(cfg, "replicas", 1) > 1 and cfg.tp == 1:
        import dataclasses as _dc

        import torch

        from ..engine.async_llm import device_guard
        from ..parallel.state import ParallelState
        n = cfg.replicas
        engines = []
        for i in range(n):
            dev = torch.device(f"cuda:{i}") if torch.cuda.is_available() else torch.device("cpu")
            ecfg = _dc.replace(EngineConfig.from_server_config(cfg), device=str(dev))
            with device_guard(dev):
                engines.append(LLMEngine(ecfg, ParallelState(device=dev)))
        llm = ReplicaPool([AsyncLLM(e) for e in engines])
        engine = engines[0]
    else:
        built = engine is None
        if built:
            st = init_parallel(tp=cfg.tp, ep=cfg.ep)
            engine = LLMEngine(EngineConfig.from_server_config(cfg), st)
            if st.tp_rank != 0:
                try:
                    engine.runner.worker_loop()  # never returns until the leader stops
                except BaseException as e:  # noqa: BLE001 - leader died / collective failed
                    logger.error("TP worker failed", error=repr(e), rank=st.rank)
                    try:
                        engine.runner.abort_comms()
                    finally:
                        from ..server.app import hard_exit
                        hard_exit(1)
                raise SystemExit(0)
        llm = AsyncLLM(engine)
        st = engine.st
        if built and st.world_size > 1 and st.tp_size == 1 and not engine.lockstep:
            # DP under torchrun (one engine per GPU rank): ONE front end on rank 0 routes to every
            # rank's engine process; the other ranks serve their engine until it stops them
            from ..engine.remote import dp_gateway
            pool = dp_gateway(llm, st)
            if pool is None:
                llm.shutdown()
                raise SystemExit(0)
            llm = pool
    name = cfg.model if isinstance(cfg.model, str) else "model"
    router.register_model_tool("llm.generate", name, LLMTool("llm.generate", name, llm, chat=False))
    chat_tool = LLMTool("llm.chat", name, llm, chat=True)
    chat_tool.router = router
    router.register_model_tool("llm.chat", name, chat_tool)
    router.llm = llm
    logger.info("local LLM backend ready", model=name, kv_blocks=engine.runner.num_blocks,
                block_size=engine.cfg.block_size, tp=engine.st.tp_size,
                replicas=len(getattr(llm, "replicas", [llm])))
    return llm
