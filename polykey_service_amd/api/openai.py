"""OpenAI-compatible HTTP route (config 4 of BASELINE.json: "70B TP=8, OpenAI-compatible chat
route").  No reference counterpart (no HTTP/OpenAI route in polykey).

Endpoints: ``POST /v1/chat/completions`` and ``POST /v1/completions`` (``stream: true`` →
server-sent events ending with ``data: [DONE]``), ``GET /v1/models``, ``GET /health``.
Chat requests accept OpenAI ``tools`` / ``tool_choice`` (calls returned as ``tool_calls`` with
``finish_reason: "tool_calls"``) plus the polykey extensions ``execute_tools`` (route the calls
to the gateway's own tools and continue the chat), ``tool_secret_id`` and ``max_tool_rounds``
(service/tool_calls.py).  A tool-enabled chat is decided whole before it is streamed, so its
SSE stream carries the content or the calls in one delta.
Requests are served by the same :class:`ToolRouter` model tools as gRPC, so both fronts share
one continuous-batching engine; ``model`` selects the backend like ``llm.chat:<model>``.
"""


import asyncio
import json
import time
import uuid
from typing import Any, Dict, List, Optional

from ..engine.sequence import SamplingParams
from ..service.base import ToolError
from ..service.tool_calls import run_chat, tool_rounds, validate_tools

_SAMPLING_KEYS = ("max_tokens", "temperature", "top_p", "top_k", "min_p", "seed", "stop", "ignore_eos",
                  "stop_token_ids", "cache_salt")



def _usage(n_prompt: int, n_out: int, metrics) -> dict:
    """OpenAI usage block; ``prompt_tokens_details.cached_tokens`` = prompt tokens whose KV came
    from the prefix cache (engine/scheduler.py)."""
    return {"prompt_tokens": n_prompt, "completion_tokens": n_out, "total_tokens": n_prompt + n_out,
            "prompt_tokens_details": {"cached_tokens": int((metrics or {}).get("cached_prompt_tokens") or 0)}}

def _llm(router, model: Optional[str]):
    """The AsyncLLM serving ``model`` (the ``llm.chat`` tool registered for it)."""
    models = router.models("llm.chat")
    if not models:
        raise ToolError("UNAVAILABLE", "no local LLM backend attached")
    if model and model not in models:
        raise ToolError("NOT_FOUND", f"model {model!r} not served; available: {models}")
    tool = router.resolve("llm.chat" + (f":{model}" if model else ""), {})
    return tool.llm, tool.model_name


def _params(body: Dict[str, Any]) -> SamplingParams:
    d = {k: body[k] for k in _SAMPLING_KEYS if k in body and body[k] is not None}
    if "max_completion_tokens" in body and "max_tokens" not in d:
        d["max_tokens"] = body["max_completion_tokens"]
    d.setdefault("max_tokens", 256)
    d.setdefault("temperature", 1.0)
    sp = SamplingParams.from_dict(d)
    sp.validate(1 << 30)
    return sp


def create_app(router):
    from fastapi import FastAPI, Request
    from fastapi.responses import JSONResponse, StreamingResponse

    app = FastAPI(title="polykey OpenAI-compatible API")

    def err(status: int, msg: str, typ: str = "invalid_request_error"):
        return JSONResponse({"error": {"message": msg, "type": typ}}, status_code=status)

    @app.get("/health")
    async def health():
        llm = getattr(router, "llm", None)
        ok = llm is None or llm.healthy()
        return JSONResponse({"status": "ok" if ok else "unhealthy"}, status_code=200 if ok else 503)

    @app.get("/v1/models")
    async def models():
        now = int(time.time())
        return {"object": "list", "data": [{"id": m, "object": "model", "created": now, "owned_by": "polykey"}
                                           for m in router.models("llm.chat")]}

    async def _run(body: Dict[str, Any], chat: bool):
        try:
            llm, model = _llm(router, body.get("model"))
            sp = _params(body)
        except ToolError as e:
            return err(404 if e.code == "NOT_FOUND" else 503, e.message)
        except (ValueError, TypeError) as e:
            return err(400, str(e))
        tok = llm.tokenizer
        if chat:
            msgs = body.get("messages")
            if not isinstance(msgs, list) or not msgs:
                return err(400, "'messages' must be a non-empty list")
            try:
                tools, choice = validate_tools(body.get("tools"), body.get("tool_choice"))
            except ValueError as e:
                return err(400, str(e))
            if tools and choice != "none":
                return await _run_tools(body, llm, model, msgs, sp, tools, choice)
            prompt_ids = tok.encode(tok.apply_chat_template(msgs))
        else:
            p = body.get("prompt")
            if isinstance(p, list) and p and isinstance(p[0], int):
                prompt_ids = [int(x) for x in p]
            elif isinstance(p, str) and p:
                prompt_ids = tok.encode(p)
            else:
                return err(400, "'prompt' must be a non-empty string or token id list")
        rid = ("chatcmpl-" if chat else "cmpl-") + uuid.uuid4().hex[:24]
        created = int(time.time())
        obj = "chat.completion" if chat else "text_completion"

        if body.get("stream"):
            async def sse():
                from ..engine.tokenizer import IncrementalDetokenizer
                toks: List[int] = []
                detok = IncrementalDetokenizer(tok)
                finish = None
                final_metrics = None
                if chat:
                    first = {"id": rid, "object": "chat.completion.chunk", "created": created, "model": model,
                             "choices": [{"index": 0, "delta": {"role": "assistant"}, "finish_reason": None}]}
                    yield f"data: {json.dumps(first)}\n\n"
                agen = llm.generate(prompt_ids, sp, request_id=rid)
                try:
                    async for out in agen:
                        toks.extend(out.new_token_ids)
                        finish = out.finish_reason
                        final_metrics = out.metrics or final_metrics
                        delta = detok.push(out.new_token_ids)
                        if delta:
                            choice = ({"index": 0, "delta": {"content": delta}, "finish_reason": None} if chat
                                      else {"index": 0, "text": delta, "finish_reason": None})
                            ch = {"id": rid, "object": obj + (".chunk" if chat else ""), "created": created,
                                  "model": model, "choices": [choice]}
                            yield f"data: {json.dumps(ch)}\n\n"
                finally:
                    await agen.aclose()
                last_choice = ({"index": 0, "delta": {}, "finish_reason": finish} if chat
                               else {"index": 0, "text": "", "finish_reason": finish})
                last = {"id": rid, "object": obj + (".chunk" if chat else ""), "created": created, "model": model,
                        "choices": [last_choice],
                        "usage": _usage(len(prompt_ids), len(toks), final_metrics)}
                yield f"data: {json.dumps(last)}\n\n"
                yield "data: [DONE]\n\n"

            return StreamingResponse(sse(), media_type="text/event-stream")

        toks, last = await llm.generate_all(prompt_ids, sp, request_id=rid)
        text = tok.decode(toks)
        if sp.stop:
            cuts = [text.find(s) for s in sp.stop if text.find(s) >= 0]
            if cuts:
                text = text[:min(cuts)]
        choice = ({"index": 0, "message": {"role": "assistant", "content": text},
                   "finish_reason": last.finish_reason if last else None} if chat
                  else {"index": 0, "text": text, "finish_reason": last.finish_reason if last else None})
        return {"id": rid, "object": obj, "created": created, "model": model, "choices": [choice],
                "usage": _usage(len(prompt_ids), len(toks), last.metrics if last else None)}

    async def _run_tools(body, llm, model, msgs, sp, tools, choice):
        rid = "chatcmpl-" + uuid.uuid4().hex[:24]
        created = int(time.time())
        try:
            rounds = tool_rounds(body.get("max_tool_rounds"))
            oc = await run_chat(llm, llm.tokenizer.chat_template, msgs, sp, tools, choice, router=router,
                                execute=bool(body.get("execute_tools")), secret_id=body.get("tool_secret_id"),
                                max_rounds=rounds, request_id=rid)
        except (ValueError, TypeError) as e:
            return err(400, str(e))
        usage = _usage(oc.prompt_tokens, oc.completion_tokens, oc.metrics)
        extra = {"polykey_tool_results": oc.executed} if oc.executed else {}
        if not body.get("stream"):
            msg = {"role": "assistant", "content": oc.content if oc.content or not oc.tool_calls else None}
            if oc.tool_calls:
                msg["tool_calls"] = oc.tool_calls
            return {"id": rid, "object": "chat.completion", "created": created, "model": model,
                    "choices": [{"index": 0, "message": msg, "finish_reason": oc.finish_reason}], "usage": usage,
                    **extra}

        async def sse():
            def chunk(delta, finish=None, **kw):
                return "data: " + json.dumps({"id": rid, "object": "chat.completion.chunk", "created": created,
                                              "model": model, "choices": [{"index": 0, "delta": delta,
                                                                           "finish_reason": finish}], **kw}) + "\n\n"
            yield chunk({"role": "assistant"})
            if oc.tool_calls:
                yield chunk({"tool_calls": [{"index": i, **c} for i, c in enumerate(oc.tool_calls)]})
            elif oc.content:
                yield chunk({"content": oc.content})
            yield chunk({}, oc.finish_reason, usage=usage, **extra)
            yield "data: [DONE]\n\n"

        return StreamingResponse(sse(), media_type="text/event-stream")

    @app.post("/v1/chat/completions")
    async def chat_completions(request: Request):
        try:
            body = await request.json()
        except json.JSONDecodeError:
            return err(400, "invalid JSON")
        return await _run(body, chat=True)

    @app.post("/v1/completions")
    async def completions(request: Request):
        try:
            body = await request.json()
        except json.JSONDecodeError:
            return err(400, "invalid JSON")
        return await _run(body, chat=False)

    return app


class _HttpHandle:
    def __init__(self, server, task):
        self.server = server
        self.task = task

    async def shutdown(self):
        self.server.should_exit = True
        await self.task


async def serve_openai(router, addr: str, logger):
    import uvicorn
    host, _, port = addr.rpartition(":")
    cfg = uvicorn.Config(create_app(router), host=host or "0.0.0.0", port=int(port), log_level="warning",
                         lifespan="off")
    server = uvicorn.Server(cfg)
    task = asyncio.create_task(server.serve())
    logger.info("openai route listening", address=addr)
    return _HttpHandle(server, task)
