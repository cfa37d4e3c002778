"""Tool calling for the chat route: parse model-emitted calls, force calls, and route calls to
the gateway's own tools.

This is the "tool-call routing path" of BASELINE.json config 5.  The reference's routing is a
dispatch on ``tool_name`` (``/root/reference/internal/service/mock.go:32-64``); here the model
itself names the tool:

1. the chat (with OpenAI ``tools``) is rendered by the family's :class:`ChatTemplate`;
2. ``tool_choice``: ``"none"`` renders no tools; a named function (or ``"required"`` with a
   single tool) appends the family's call opening to the prompt so the completion *is* that
   call's arguments; ``"required"`` with several tools opens a call and lets the model pick
   the name; ``"auto"`` parses calls out of free text (:func:`parse_tool_calls`);
3. with ``execute_tools`` (a polykey extension, OpenAI and gRPC alike) every parsed call whose
   name the :class:`~polykey_service_amd.service.router.ToolRouter` serves -- the mock tools,
   secret-gated tools (``tool_secret_id``), anything registered -- is executed through the
   router, its result appended as a ``tool`` message, and the model runs again (up to
   ``max_tool_rounds``); model tools (``llm.*``) are never called recursively.

OpenAI semantics kept: ``arguments`` is a JSON string (the model's own text when it did not
produce valid JSON, as OpenAI documents), ``finish_reason`` is ``"tool_calls"`` when calls
are returned to the client.
"""
from __future__ import annotations

import dataclasses
import json
import os
import uuid
from typing import Any, Dict, List, Optional, Tuple

from ..engine.chat_template import MISTRAL, ChatTemplate

_DEC = json.JSONDecoder()
_END_MARKERS = ("<|eom_id|>", "<|eot_id|>", "</s>", "<|end_of_text|>")


def _call(name: str, args: Any) -> Dict[str, Any]:
    if not isinstance(args, str):
        args = json.dumps(args if args is not None else {}, ensure_ascii=False)
    return {"id": "call_" + uuid.uuid4().hex[:24], "type": "function", "function": {"name": name, "arguments": args}}


def _from_obj(o: Any) -> Optional[Dict[str, Any]]:
    if isinstance(o, dict) and isinstance(o.get("name"), str) and o["name"]:
        args = o.get("arguments", o.get("parameters", {}))
        return _call(o["name"], args)
    return None


def _strip_end(s: str) -> str:
    for m in _END_MARKERS:
        s = s.replace(m, "")
    return s.strip()


def _json_seq(s: str) -> Tuple[List[Any], str]:
    """Consecutive JSON values at the start of ``s`` (separated by whitespace , or ;) and the
    unparsed rest."""
    vals = []
    i = 0
    while True:
        while i < len(s) and s[i] in " \t\r\n,;":
            i += 1
        if i >= len(s) or s[i] not in "{[":
            break
        try:
            v, i = _DEC.raw_decode(s, i)
        except json.JSONDecodeError:
            break
        vals.append(v)
    return vals, s[i:]


def parse_tool_calls(text: str, allowed: Optional[List[str]] = None) -> Tuple[str, List[Dict[str, Any]]]:
    """→ (content, tool_calls).  Recognised: ``[TOOL_CALLS] [...]`` (Mistral), ``<tool_call>
    {...}</tool_call>`` blocks, and a reply that is one or more JSON call objects (Llama-3,
    optionally after ``<|python_tag|>``).  Calls naming a function not in ``allowed`` are
    dropped; if nothing valid remains the whole text is content."""
    s = _strip_end(text)
    calls: List[Dict[str, Any]] = []
    content = s
    if "[TOOL_CALLS]" in s:
        content, _, rest = s.partition("[TOOL_CALLS]")
        vals, _ = _json_seq(rest.strip())
        for v in vals:
            for o in (v if isinstance(v, list) else [v]):
                c = _from_obj(o)
                if c:
                    calls.append(c)
    elif "<tool_call>" in s:
        content = s[:s.index("<tool_call>")]
        for block in s.split("<tool_call>")[1:]:
            vals, _ = _json_seq(block.split("</tool_call>")[0].strip())
            for v in vals:
                c = _from_obj(v)
                if c:
                    calls.append(c)
    else:
        body = s[len("<|python_tag|>"):] if s.startswith("<|python_tag|>") else s
        vals, rest = _json_seq(body)
        objs = [c for c in (_from_obj(v) for v in vals)]
        if vals and all(objs) and not rest.strip():
            calls, content = objs, ""
    if allowed is not None:
        calls = [c for c in calls if c["function"]["name"] in allowed]
    if not calls:
        return s, []
    return content.strip(), calls


def forced_call(generated: str, name: Optional[str], allowed: List[str], family: str) -> Dict[str, Any]:
    """The call a forced prompt (``ChatTemplate.call_prefix``) produced: ``generated`` continues
    the opening, so for a named call it starts with the arguments."""
    g = _strip_end(generated)
    if name is None:  # the model wrote the name: re-assemble the whole call and parse it
        opening = '[{"name": "' if family == MISTRAL else '{"name": "'
        _, calls = parse_tool_calls(("[TOOL_CALLS] " if family == MISTRAL else "") + opening + g, allowed)
        if calls:
            return calls[0]
        # no parseable call: the offered name the text starts with, else the first offered one
        name = max((n for n in allowed if g.startswith(n)), key=len, default=allowed[0])
        g = g[len(name):].lstrip('"').lstrip(", ").partition(":")[2].strip() if g.startswith(name) else g
    try:
        args, _ = _DEC.raw_decode(g.lstrip())
        return _call(name, args)
    except json.JSONDecodeError:
        raw = g.rstrip()
        for tail in ("}]", "}"):  # the call object's own closing
            if raw.endswith(tail) and raw.count("{") < raw.count("}"):
                raw = raw[:-len(tail)].rstrip()
                break
        return _call(name, raw)


# server-side cap on client-requested tool rounds (each round is a full generation that may run
# gateway tools with model-written arguments)
MAX_TOOL_ROUNDS = int(os.environ.get("POLYKEY_MAX_TOOL_ROUNDS", "8"))


def tool_rounds(value: Any, default: int = 3, cap: Optional[int] = None) -> int:
    """Validate a client's ``max_tool_rounds``: an integer >= 1, clamped to the server cap."""
    if value is None:
        value = default
    if isinstance(value, bool) or not isinstance(value, (int, float)) or int(value) != value:
        raise ValueError("max_tool_rounds must be an integer")
    if value < 1:
        raise ValueError("max_tool_rounds must be >= 1")
    return min(int(value), MAX_TOOL_ROUNDS if cap is None else cap)


def tool_names(tools: Optional[List[Dict[str, Any]]]) -> List[str]:
    out = []
    for t in tools or []:
        fn = t.get("function", t) if isinstance(t, dict) else {}
        if isinstance(fn, dict) and fn.get("name"):
            out.append(fn["name"])
    return out


def validate_tools(tools: Any, tool_choice: Any) -> Tuple[Optional[List[Dict[str, Any]]], Any]:
    if tools is not None and not isinstance(tools, list):
        raise ValueError("'tools' must be a list")
    names = tool_names(tools)
    if tools and len(names) != len(tools):
        raise ValueError("every tool needs a function with a name")
    if tool_choice is None:
        tool_choice = "auto" if names else "none"
    if isinstance(tool_choice, dict):
        fn = tool_choice.get("function", {}) if isinstance(tool_choice.get("function"), dict) else {}
        if fn.get("name") not in names:
            raise ValueError(f"tool_choice names an unknown function: {fn.get('name')!r}")
    elif tool_choice not in ("none", "auto", "required"):
        raise ValueError("tool_choice must be 'none', 'auto', 'required' or a named function")
    if tool_choice == "required" and not names:
        raise ValueError("tool_choice 'required' needs tools")
    return (tools or None), tool_choice


@dataclasses.dataclass
class ChatOutcome:
    content: str
    tool_calls: List[Dict[str, Any]]
    finish_reason: Optional[str]
    prompt_tokens: int
    completion_tokens: int
    metrics: Optional[dict]
    executed: List[Dict[str, Any]]
    messages: List[Dict[str, Any]]


def _result_text(resp) -> Tuple[str, int]:
    which = resp.WhichOneof("output")
    if which == "string_output":
        text = resp.string_output
    elif which == "struct_output":
        from .. import proto
        text = json.dumps(proto.struct_to_dict(resp.struct_output), ensure_ascii=False, sort_keys=True)
    else:
        text = ""
    return text, int(resp.status.code) if resp.HasField("status") else 200


async def execute_call(router, call: Dict[str, Any], secret_id: Optional[str], request_id: str) -> Dict[str, Any]:
    """Route one model-emitted call to the gateway's tool of that name."""
    from .. import proto
    from .base import RequestContext, ToolError
    name = call["function"]["name"]
    try:
        args = json.loads(call["function"]["arguments"] or "{}")
    except json.JSONDecodeError:
        args = None
    rec = {"tool_call_id": call["id"], "name": name}
    if not isinstance(args, dict):
        return {**rec, "status": 400, "content": "error: arguments are not a JSON object"}
    params = proto.Struct()
    params.update(args)
    try:
        resp = await router.execute_tool(RequestContext(request_id=f"{request_id}:{call['id']}"), name, params,
                                         secret_id, None)
        text, code = _result_text(resp)
        return {**rec, "status": code, "content": text}
    except ToolError as e:
        return {**rec, "status": e.code, "content": f"error: {e.message}"}


def executable(router, name: str) -> bool:
    """A call the gateway may run itself: a registered tool that is not a model tool."""
    if router is None or name.partition(":")[0] in getattr(router, "_families", {}):
        return False
    return name in getattr(router, "_tools", {})


async def run_chat(llm, template: ChatTemplate, messages: List[Dict[str, Any]], sp, tools=None, tool_choice="auto",
                   router=None, execute: bool = False, secret_id: Optional[str] = None, max_rounds: int = 3,
                   request_id: Optional[str] = None) -> ChatOutcome:
    """One chat completion with tools (see the module docstring)."""
    tok = llm.tokenizer
    rid = request_id or uuid.uuid4().hex
    msgs = list(messages)
    names = tool_names(tools)
    n_prompt = n_out = 0
    executed: List[Dict[str, Any]] = []
    choice = tool_choice
    last = None
    for rnd in range(max(1, max_rounds)):
        active = bool(names) and choice != "none"
        text = template.render(msgs, tools if active else None)
        forced = False
        forced_name = None
        if active and (isinstance(choice, dict) or choice == "required"):
            forced = True
            forced_name = choice["function"]["name"] if isinstance(choice, dict) else (
                names[0] if len(names) == 1 else None)
            text += template.call_prefix(forced_name)
        prompt_ids = tok.encode(text)
        toks, last = await llm.generate_all(prompt_ids, sp, request_id=f"{rid}-{rnd}" if rnd else rid)
        n_prompt += len(prompt_ids)
        n_out += len(toks)
        out = tok.decode(toks, keep_special=active)
        if sp.stop:
            cuts = [out.find(s) for s in sp.stop if out.find(s) >= 0]
            if cuts:
                out = out[:min(cuts)]
        if forced:
            content, calls = "", [forced_call(out, forced_name, names, template.family)]
        elif active:
            content, calls = parse_tool_calls(out, names)
        else:
            content, calls = out, []
        runnable = [c for c in calls if execute and executable(router, c["function"]["name"])]
        if not calls or not runnable or len(runnable) != len(calls):
            return ChatOutcome(content, calls, "tool_calls" if calls else (last.finish_reason if last else None),
                               n_prompt, n_out, last.metrics if last else None, executed, msgs)
        msgs.append({"role": "assistant", "content": content or None, "tool_calls": calls})
        for c in calls:
            res = await execute_call(router, c, secret_id, rid)
            executed.append(res)
            msgs.append({"role": "tool", "tool_call_id": c["id"], "name": res["name"], "content": res["content"]})
        choice = "auto"  # a forced choice applies to the first turn only
    return ChatOutcome(content, [], last.finish_reason if last else None, n_prompt, n_out,
                       last.metrics if last else None, executed, msgs)
