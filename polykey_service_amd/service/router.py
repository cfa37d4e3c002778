"""Tool router: the "OpenRouter-esque" dispatch the reference promises (``README.md:27``)
but implements only as a ``switch`` inside ``MockService`` (``internal/service/mock.go:32-64``).

Resolution order for a ``tool_name``:

1. an exact registered tool (the three mock tools are always registered, so the reference's
   outputs are preserved byte for byte);
2. ``<family>:<model>`` — e.g. ``llm.chat:mixtral-8x7b`` routes to the ``llm.chat`` tool of
   the named model backend; ``llm.chat`` alone uses ``parameters.model`` or the default
   backend;
3. otherwise the reference's fallback ``"Unknown tool: <name>"`` with status 200
   (``mock.go:60-63``).

``secret_id`` (ignored by the reference mock) is resolved through an optional
:class:`~polykey_service_amd.adapters.security.secret_store.SecretStore` for tools that
declare ``requires_secret``; the plaintext never leaves the process.
"""
from __future__ import annotations

from typing import AsyncIterator, Callable, Dict, List, Optional, Protocol

from .. import proto
from .base import RequestContext, ToolError
from .mock import MOCK_TOOLS, mock_response


class Tool(Protocol):
    name: str
    requires_secret: bool

    async def run(self, ctx: RequestContext, params: dict, secret: Optional[bytes],
                  metadata: Dict[str, str]) -> "proto.ExecuteToolResponse": ...

    def stream(self, ctx: RequestContext, params: dict, secret: Optional[bytes],
               metadata: Dict[str, str]) -> AsyncIterator["proto.ExecuteToolResponse"]: ...


class _MockTool:
    requires_secret = False

    def __init__(self, name: str):
        self.name = name

    async def run(self, ctx, params, secret, metadata):
        return mock_response(self.name)

    async def stream(self, ctx, params, secret, metadata):
        yield mock_response(self.name)


class ToolRouter:
    """Implements the :class:`~polykey_service_amd.service.base.Service` protocol."""

    def __init__(self, secret_store=None):
        self._tools: Dict[str, Tool] = {}
        self._families: Dict[str, Dict[str, Tool]] = {}
        self._default_model: Dict[str, str] = {}
        self.secret_store = secret_store
        for name in MOCK_TOOLS:
            self.register(_MockTool(name))

    # ------------------------------------------------------------------ registry
    def register(self, tool: Tool) -> None:
        self._tools[tool.name] = tool

    def register_model_tool(self, family: str, model: str, tool: Tool, default: bool = False) -> None:
        self._families.setdefault(family, {})[model] = tool
        if default or family not in self._default_model:
            self._default_model[family] = model

    def tools(self) -> List[str]:
        names = list(self._tools)
        for fam, models in self._families.items():
            names.append(fam)
            names.extend(f"{fam}:{m}" for m in models)
        return names

    def models(self, family: str = "llm.chat") -> List[str]:
        return list(self._families.get(family, {}))

    def resolve(self, tool_name: str, params: dict) -> Optional[Tool]:
        if tool_name in self._tools:
            return self._tools[tool_name]
        fam, sep, model = tool_name.partition(":")
        if fam in self._families:
            models = self._families[fam]
            if not sep:
                model = str(params.get("model") or self._default_model[fam])
            if model not in models:
                raise ToolError("NOT_FOUND", f"model {model!r} is not served by tool family {fam!r}; "
                                             f"available: {sorted(models)}")
            return models[model]
        return None

    async def aclose(self) -> None:
        llm = getattr(self, "llm", None)
        if llm is not None:
            await llm.aclose()

    # ----------------------------------------------------------------- execution
    def _prepare(self, tool_name, parameters, secret_id, metadata):
        params = proto.struct_to_dict(parameters) if parameters is not None else {}
        md = dict(metadata.fields) if metadata is not None else {}
        tool = self.resolve(tool_name, params)
        secret = None
        if tool is not None and getattr(tool, "requires_secret", False):
            if secret_id is None:
                raise ToolError("UNAUTHENTICATED", f"tool {tool_name!r} requires secret_id")
            if self.secret_store is None:
                raise ToolError("FAILED_PRECONDITION", "no secret store configured")
            secret = self.secret_store.get(secret_id)
            if secret is None:
                raise ToolError("NOT_FOUND", f"secret {secret_id!r} not found")
        return tool, params, secret, md

    async def execute_tool(self, ctx: RequestContext, tool_name: str, parameters=None,
                           secret_id: Optional[str] = None, metadata=None):
        tool, params, secret, md = self._prepare(tool_name, parameters, secret_id, metadata)
        if tool is None:
            return mock_response(tool_name)  # "Unknown tool: <name>" (mock.go:60-63)
        return await tool.run(ctx, params, secret, md)

    async def execute_tool_stream(self, ctx: RequestContext, tool_name: str, parameters=None,
                                  secret_id: Optional[str] = None, metadata=None):
        tool, params, secret, md = self._prepare(tool_name, parameters, secret_id, metadata)
        if tool is None:
            yield mock_response(tool_name)
            return
        async for chunk in tool.stream(ctx, params, secret, md):
            yield chunk


def make_default_router(secret_store=None, extra: Optional[Callable[[ToolRouter], None]] = None) -> ToolRouter:
    r = ToolRouter(secret_store)
    if extra:
        extra(r)
    return r
