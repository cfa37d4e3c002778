"""Chat templates and tool-call formats for the served model families.

The reference only routes by tool name (``/root/reference/internal/service/mock.go:32-64``,
advertised as "OpenRouter-esque", ``/root/reference/README.md:27``); an on-node model has to
turn a chat (with optional function tools) into one prompt and its completion back into
either text or tool calls.  Two families are built in, matching the north-star models:

* ``llama3`` (Llama-3 8B / 70B): header-delimited turns ending in ``<|eot_id|>``; tools are
  described as JSON schemas in the system turn and a call is a JSON object
  ``{"name": ..., "parameters": {...}}``, optionally after ``<|python_tag|>``; tool results
  come back in ``ipython`` turns;
* ``mistral`` (Mixtral-8x7B): ``[INST] ... [/INST]`` turns; tools in
  ``[AVAILABLE_TOOLS] [...] [/AVAILABLE_TOOLS]`` before the last user turn; a call is
  ``[TOOL_CALLS] [{"name": ..., "arguments": {...}}, ...]`` and results are
  ``[TOOL_RESULTS] {...} [/TOOL_RESULTS]``.

When a local tokenizer directory carries a ``tokenizer_config.json`` with a ``chat_template``,
that Jinja template is rendered instead (sandboxed: no attribute access to Python internals)
and the call format is inferred from its markers.  The BOS token is not part of the rendered
text: the tokenizer adds it.
"""
from __future__ import annotations

import json
import os
from typing import Any, Dict, List, Optional

LLAMA3 = "llama3"
MISTRAL = "mistral"


def _content(m: Dict[str, Any]) -> str:
    c = m.get("content")
    if c is None:
        return ""
    if isinstance(c, list):  # OpenAI content parts: keep the text ones
        return "".join(p.get("text", "") for p in c if isinstance(p, dict) and p.get("type", "text") == "text")
    return str(c)


def _call_args(call: Dict[str, Any]) -> Any:
    fn = call.get("function", call)
    args = fn.get("arguments", fn.get("parameters", {}))
    if isinstance(args, str):
        try:
            return json.loads(args)
        except json.JSONDecodeError:
            return args
    return args


def _fn_specs(tools: Optional[List[Dict[str, Any]]]) -> List[Dict[str, Any]]:
    out = []
    for t in tools or []:
        fn = t.get("function", t) if isinstance(t, dict) else None
        if isinstance(fn, dict) and fn.get("name"):
            out.append({"type": "function", "function": {k: fn[k] for k in ("name", "description", "parameters")
                                                           if k in fn}})
    return out


class ChatTemplate:
    """``render(messages, tools)`` → prompt text; ``call_prefix(name)`` → the text that opens a
    call to ``name`` (``name=None``: a call to a function the model picks) in this family's
    format, appended to the prompt to force a tool call."""

    def __init__(self, family: str = LLAMA3, jinja_source: Optional[str] = None, special: Optional[dict] = None):
        self.family = family
        self.jinja_source = jinja_source
        self.special = special or {}
        self._jinja = None
        if jinja_source:
            from jinja2.sandbox import ImmutableSandboxedEnvironment
            env = ImmutableSandboxedEnvironment(trim_blocks=True, lstrip_blocks=True)

            def raise_exception(msg):
                raise ValueError(msg)

            env.globals["raise_exception"] = raise_exception
            env.filters["tojson"] = lambda v, indent=None: json.dumps(v, indent=indent, ensure_ascii=False)
            self._jinja = env.from_string(jinja_source)

    # ------------------------------------------------------------------ render
    def render(self, messages: List[Dict[str, Any]], tools: Optional[List[Dict[str, Any]]] = None,
               add_generation_prompt: bool = True) -> str:
        specs = _fn_specs(tools)
        if self._jinja is not None:
            text = self._jinja.render(messages=messages, tools=specs or None, add_generation_prompt=add_generation_prompt,
                                      bos_token="", eos_token=self.special.get("eos_token", ""))
            return text
        if self.family == MISTRAL:
            return self._render_mistral(messages, specs)
        return self._render_llama3(messages, specs, add_generation_prompt)

    def _render_llama3(self, messages, specs, add_generation_prompt) -> str:
        def turn(role: str, body: str, end: str = "<|eot_id|>") -> str:
            return f"<|start_header_id|>{role}<|end_header_id|>\n\n{body}{end}"

        parts = []
        msgs = list(messages)
        system = ""
        if msgs and msgs[0].get("role") == "system":
            system = _content(msgs.pop(0))
        if specs:
            tool_text = ("You can call functions. To call one, reply with only a JSON object of the form "
                         '{"name": <function name>, "parameters": <object of argument values>}. '
                         "Available functions:\n" + "\n".join(json.dumps(s, ensure_ascii=False) for s in specs))
            system = (system + "\n\n" + tool_text) if system else tool_text
            system = "Environment: ipython\n" + system
        if system:
            parts.append(turn("system", system))
        for m in msgs:
            role = m.get("role", "user")
            if role == "assistant" and m.get("tool_calls"):
                calls = "; ".join(json.dumps({"name": c.get("function", c).get("name"), "parameters": _call_args(c)},
                                             ensure_ascii=False) for c in m["tool_calls"])
                parts.append(turn("assistant", "<|python_tag|>" + calls, "<|eom_id|>"))
            elif role in ("tool", "ipython"):
                parts.append(turn("ipython", _content(m)))
            else:
                parts.append(turn(role, _content(m)))
        if add_generation_prompt:
            parts.append("<|start_header_id|>assistant<|end_header_id|>\n\n")
        return "".join(parts)

    def _render_mistral(self, messages, specs) -> str:
        parts = []
        msgs = list(messages)
        system = ""
        if msgs and msgs[0].get("role") == "system":
            system = _content(msgs.pop(0))
        last_user = max((i for i, m in enumerate(msgs) if m.get("role", "user") == "user"), default=-1)
        for i, m in enumerate(msgs):
            role = m.get("role", "user")
            if role == "user":
                if specs and i == last_user:
                    parts.append("[AVAILABLE_TOOLS] " + json.dumps(specs, ensure_ascii=False) + "[/AVAILABLE_TOOLS]")
                body = _content(m)
                if system and i == last_user:
                    body = system + "\n\n" + body
                parts.append(f"[INST] {body} [/INST]")
            elif role == "assistant":
                if m.get("tool_calls"):
                    calls = [{"name": c.get("function", c).get("name"), "arguments": _call_args(c)}
                             for c in m["tool_calls"]]
                    parts.append("[TOOL_CALLS] " + json.dumps(calls, ensure_ascii=False) + "</s>")
                else:
                    parts.append(_content(m) + "</s>")
            elif role in ("tool", "ipython"):
                res = {"content": _content(m)}
                if m.get("tool_call_id"):
                    res["call_id"] = m["tool_call_id"]
                parts.append("[TOOL_RESULTS] " + json.dumps(res, ensure_ascii=False) + "[/TOOL_RESULTS]")
        return "".join(parts)

    # ------------------------------------------------------------- forced calls
    def call_prefix(self, name: Optional[str]) -> str:
        if self.family == MISTRAL:
            return '[TOOL_CALLS] [{"name": "' + (f'{name}", "arguments": ' if name else "")
        return '<|python_tag|>{"name": "' + (f'{name}", "parameters": ' if name else "")


def family_for(model_name: str, is_moe: bool = False) -> str:
    n = (model_name or "").lower()
    return MISTRAL if is_moe or "mixtral" in n or "mistral" in n else LLAMA3


def load_chat_template(tokenizer_dir: str, family: str) -> ChatTemplate:
    """The tokenizer directory's Jinja chat template when it has one (call format inferred from
    its markers), else the built-in template of ``family``."""
    cfg_path = os.path.join(tokenizer_dir, "tokenizer_config.json") if tokenizer_dir else ""
    if cfg_path and os.path.isfile(cfg_path):
        with open(cfg_path) as f:
            tc = json.load(f)
        src = tc.get("chat_template")
        if isinstance(src, list):  # named templates: take "default"
            src = next((t.get("template") for t in src if t.get("name") == "default"), None)
        if isinstance(src, str) and src:
            fam = MISTRAL if "[TOOL_CALLS]" in src or "[INST]" in src else (
                LLAMA3 if "<|start_header_id|>" in src else family)
            eos = tc.get("eos_token")
            eos = eos.get("content") if isinstance(eos, dict) else eos
            return ChatTemplate(fam, jinja_source=src, special={"eos_token": eos or ""})
    return ChatTemplate(family)
