"""L2 RPC adapter: ``polykey.v2.PolykeyService`` → :class:`Service` call.

Reference ``internal/server/server.go:12-43``:

* logs ``"ExecuteTool called" {tool_name, has_parameters, has_secret_id, has_metadata}``
  (``server.go:28-33``) — here through the same JSON logger as the interceptor (the
  reference used ``slog.Default()``'s text handler by accident);
* forwards the unpacked fields to the service (``server.go:36``), ``secret_id`` as ``None``
  when the proto3-optional field is unset (Go ``*string`` nil);
* on error logs ``"Service ExecuteTool failed" {error}`` and returns it (``server.go:37-40``):
  a :class:`ToolError` keeps its status code, anything else is ``UNKNOWN`` like a raw Go error.

Every other method of the service is UNIMPLEMENTED (the Go struct embeds
``UnimplementedPolykeyServiceServer``, ``server.go:13``); grpc does that for unknown methods.
[NEW] ``ExecuteToolStream`` streams partial outputs and propagates client cancellation into the
service (the engine frees KV blocks of an abandoned request).
"""
from __future__ import annotations

import asyncio
import time

import grpc

from .. import proto
from ..service.base import RequestContext, ToolError
from ..utils import slog


def _ctx_from_grpc(context) -> RequestContext:
    remaining = None
    try:
        remaining = context.time_remaining()
    except Exception:
        pass
    deadline = None if remaining is None else time.monotonic() + remaining
    rid = None
    try:
        for k, v in context.invocation_metadata() or ():
            if k == "x-request-id":
                rid = v
    except Exception:
        pass
    peer = ""
    try:
        peer = context.peer()
    except Exception:
        pass
    return RequestContext(deadline=deadline, request_id=rid, peer=peer)


class PolykeyServicer:
    def __init__(self, service, logger: slog.Logger):
        self.service = service
        self.logger = logger

    def _log_call(self, method: str, req) -> None:
        self.logger.info(f"{method} called",
                         tool_name=req.tool_name,
                         has_parameters=req.HasField("parameters"),
                         has_secret_id=req.HasField("secret_id"),
                         has_metadata=req.HasField("metadata"))

    @staticmethod
    def _unpack(req):
        return (req.tool_name,
                req.parameters if req.HasField("parameters") else None,
                req.secret_id if req.HasField("secret_id") else None,
                req.metadata if req.HasField("metadata") else None)

    async def _fail(self, method: str, context, e: BaseException):
        self.logger.error(f"Service {method} failed", error=str(e))
        if isinstance(e, ToolError):
            await context.abort(getattr(grpc.StatusCode, e.code, grpc.StatusCode.UNKNOWN), e.message)
        await context.abort(grpc.StatusCode.UNKNOWN, str(e))

    async def ExecuteTool(self, request, context):
        self._log_call("ExecuteTool", request)
        ctx = _ctx_from_grpc(context)
        try:
            return await self.service.execute_tool(ctx, *self._unpack(request))
        except asyncio.CancelledError:
            ctx.cancel()
            raise
        except grpc.aio.AbortError:
            raise
        except Exception as e:  # noqa: BLE001
            await self._fail("ExecuteTool", context, e)

    async def ExecuteToolStream(self, request, context):
        self._log_call("ExecuteToolStream", request)
        ctx = _ctx_from_grpc(context)
        agen = self.service.execute_tool_stream(ctx, *self._unpack(request))
        try:
            async for chunk in agen:
                yield chunk
        except asyncio.CancelledError:
            ctx.cancel()
            raise
        except grpc.aio.AbortError:
            raise
        except Exception as e:  # noqa: BLE001
            await self._fail("ExecuteToolStream", context, e)
        finally:
            ctx.cancel()
            await agen.aclose()

    def handler(self) -> grpc.GenericRpcHandler:
        ser = proto.ExecuteToolResponse.SerializeToString
        de = proto.ExecuteToolRequest.FromString
        return grpc.method_handlers_generic_handler(proto.POLYKEY_SERVICE, {
            "ExecuteTool": grpc.unary_unary_rpc_method_handler(
                self.ExecuteTool, request_deserializer=de, response_serializer=ser),
            "ExecuteToolStream": grpc.unary_stream_rpc_method_handler(
                self.ExecuteToolStream, request_deserializer=de, response_serializer=ser),
        })


SERVICE_METHODS = {
    proto.POLYKEY_SERVICE: ["ExecuteTool", "ExecuteToolStream"],
    proto.HEALTH_SERVICE: ["Check", "Watch"],
    "grpc.reflection.v1alpha.ServerReflection": ["ServerReflectionInfo"],
    "grpc.reflection.v1.ServerReflection": ["ServerReflectionInfo"],
}
