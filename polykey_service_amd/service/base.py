"""The service seam between the RPC layer and backends.

Reference: ``internal/service/service.go:12-15`` — one method
``ExecuteTool(ctx, toolName, *structpb.Struct, *string, *cmn.Metadata)``.  The Python
protocol keeps that signature (``secret_id`` is ``None`` when the proto3-optional field is
unset, like the Go ``*string``) and adds the streaming variant used by the new
``ExecuteToolStream`` RPC.
"""
from __future__ import annotations

import asyncio
import time
import uuid
from typing import AsyncIterator, Optional, Protocol, runtime_checkable

from .. import proto


class ToolError(Exception):
    """An error with a gRPC status code (maps onto ``status.Error`` in Go)."""

    def __init__(self, code: str, message: str):
        super().__init__(message)
        self.code = code  # grpc.StatusCode name, e.g. "INVALID_ARGUMENT"
        self.message = message


class RequestContext:
    """Per-call context (Go's ``context.Context`` analogue): deadline + cancellation."""

    def __init__(self, deadline: Optional[float] = None, request_id: Optional[str] = None,
                 peer: str = ""):
        self.deadline = deadline  # absolute time.monotonic() or None
        self.request_id = request_id or uuid.uuid4().hex
        self.peer = peer
        self.cancelled = asyncio.Event() if _has_loop() else None
        self.start = time.monotonic()

    def time_remaining(self) -> Optional[float]:
        return None if self.deadline is None else self.deadline - time.monotonic()

    def cancel(self) -> None:
        if self.cancelled is not None:
            self.cancelled.set()

    def is_cancelled(self) -> bool:
        return self.cancelled is not None and self.cancelled.is_set()


def _has_loop() -> bool:
    try:
        asyncio.get_running_loop()
        return True
    except RuntimeError:
        return False


@runtime_checkable
class Service(Protocol):
    async def execute_tool(self, ctx: RequestContext, tool_name: str, parameters: Optional["proto.Struct"],
                           secret_id: Optional[str], metadata: Optional["proto.Metadata"]) -> "proto.ExecuteToolResponse":
        ...

    def execute_tool_stream(self, ctx: RequestContext, tool_name: str, parameters: Optional["proto.Struct"],
                            secret_id: Optional[str], metadata: Optional["proto.Metadata"]
                            ) -> AsyncIterator["proto.ExecuteToolResponse"]:
        ...


def ok_status(message: str = "Tool executed successfully"):
    return proto.Status(code=200, message=message)
