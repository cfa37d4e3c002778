"""Logging interceptor with the reference's log schema (``cmd/polykey/main.go:25-52``).

* ``/grpc.health.v1.Health/Check`` bypasses logging (``main.go:29-31``)
* ``"gRPC call received" {method}`` before the handler (``main.go:33``)
* ``"gRPC call finished" {method, duration, code}`` after it, INFO on success and ERROR on
  failure (``main.go:37-48``); ``duration`` is Go's ``Duration.String()`` and ``code`` Go's
  ``codes.Code.String()`` so R17/R18-style consumers parse it unchanged.

[NEW] The reference intercepts unary calls only; this interceptor also wraps server-streaming
and bidi handlers (same schema) and adds a ``request_id`` attribute so a log consumer can key
concurrent calls of one method apart.  An optional ``observer`` gets
``(method, seconds, code)`` for metrics.
"""
from __future__ import annotations

import itertools
import time
from typing import Callable, Optional

import grpc

from ..utils import slog

GO_CODE = {
    "OK": "OK", "CANCELLED": "Canceled", "UNKNOWN": "Unknown", "INVALID_ARGUMENT": "InvalidArgument",
    "DEADLINE_EXCEEDED": "DeadlineExceeded", "NOT_FOUND": "NotFound", "ALREADY_EXISTS": "AlreadyExists",
    "PERMISSION_DENIED": "PermissionDenied", "RESOURCE_EXHAUSTED": "ResourceExhausted",
    "FAILED_PRECONDITION": "FailedPrecondition", "ABORTED": "Aborted", "OUT_OF_RANGE": "OutOfRange",
    "UNIMPLEMENTED": "Unimplemented", "INTERNAL": "Internal", "UNAVAILABLE": "Unavailable",
    "DATA_LOSS": "DataLoss", "UNAUTHENTICATED": "Unauthenticated",
}

HEALTH_CHECK = "/grpc.health.v1.Health/Check"
_ids = itertools.count(1)


def _final_code(context, exc: Optional[BaseException]) -> str:
    code = None
    try:
        code = context.code()
    except Exception:
        code = None
    if code is None or code == grpc.StatusCode.OK:
        if exc is None:
            return "OK"
        if isinstance(exc, grpc.aio.AbortError) and code is not None:
            return GO_CODE.get(code.name, "Unknown")
        import asyncio
        if isinstance(exc, asyncio.CancelledError):
            return "Canceled"
        return "Unknown"
    return GO_CODE.get(code.name, "Unknown") if hasattr(code, "name") else "Unknown"


class LoggingInterceptor(grpc.aio.ServerInterceptor):
    def __init__(self, logger: slog.Logger, observer: Optional[Callable[[str, float, str], None]] = None):
        self.logger = logger
        self.observer = observer

    def _begin(self, method: str) -> int:
        rid = next(_ids)
        self.logger.info("gRPC call received", method=method, request_id=rid)
        return rid

    def _end(self, method: str, rid: int, t0: float, context, exc) -> None:
        dt = time.perf_counter() - t0
        code = _final_code(context, exc)
        level = slog.INFO if code == "OK" else slog.ERROR
        self.logger.log(level, "gRPC call finished", method=method, duration=slog.go_duration(dt),
                        code=code, request_id=rid)
        if self.observer is not None:
            try:
                self.observer(method, dt, code)
            except Exception:
                pass

    async def intercept_service(self, continuation, handler_call_details):
        handler = await continuation(handler_call_details)
        method = handler_call_details.method
        if handler is None or method == HEALTH_CHECK:
            return handler

        if handler.unary_unary is not None:
            inner = handler.unary_unary

            async def unary_unary(request, context):
                t0 = time.perf_counter()
                rid = self._begin(method)
                exc = None
                try:
                    return await inner(request, context)
                except BaseException as e:  # noqa: BLE001 - re-raised
                    exc = e
                    raise
                finally:
                    self._end(method, rid, t0, context, exc)

            return handler._replace(unary_unary=unary_unary)

        if handler.unary_stream is not None:
            inner_s = handler.unary_stream

            async def unary_stream(request, context):
                t0 = time.perf_counter()
                rid = self._begin(method)
                exc = None
                try:
                    async for item in inner_s(request, context):
                        yield item
                except BaseException as e:  # noqa: BLE001
                    exc = e
                    raise
                finally:
                    self._end(method, rid, t0, context, exc)

            return handler._replace(unary_stream=unary_stream)

        if handler.stream_stream is not None:
            inner_ss = handler.stream_stream

            async def stream_stream(request_iterator, context):
                t0 = time.perf_counter()
                rid = self._begin(method)
                exc = None
                try:
                    async for item in inner_ss(request_iterator, context):
                        yield item
                except BaseException as e:  # noqa: BLE001
                    exc = e
                    raise
                finally:
                    self._end(method, rid, t0, context, exc)

            return handler._replace(stream_stream=stream_stream)

        return handler
