"""``grpc.health.v1.Health`` implemented on grpc.aio (the python health package is absent).

Reference behaviour (``cmd/polykey/main.go:82,90,93-94,118``): SERVING for
``"polykey.v2.PolykeyService"`` and ``""``; ``Shutdown()`` flips every service to
NOT_SERVING and ignores later updates.  ``Check`` of an unknown service returns
NOT_FOUND, ``Watch`` of one streams SERVICE_UNKNOWN, as grpc-go's health server does.
[NEW] the engine's watchdog calls :meth:`set_serving_status` to report NOT_SERVING when the
engine loop dies.
"""
from __future__ import annotations

import asyncio
from typing import Dict, Set

import grpc

from .. import proto

SS = proto.HealthCheckResponse.ServingStatus
SERVING = SS.Value("SERVING")
NOT_SERVING = SS.Value("NOT_SERVING")
SERVICE_UNKNOWN = SS.Value("SERVICE_UNKNOWN")


class HealthServicer:
    def __init__(self):
        self._status: Dict[str, int] = {}
        self._watchers: Dict[str, Set[asyncio.Queue]] = {}
        self._shutdown = False

    def set_serving_status(self, service: str, status: int) -> None:
        if self._shutdown:
            return
        self._set(service, status)

    def _set(self, service: str, status: int) -> None:
        self._status[service] = status
        for q in list(self._watchers.get(service, ())):
            q.put_nowait(status)

    def get(self, service: str):
        return self._status.get(service)

    def shutdown(self) -> None:
        """Flip everything to NOT_SERVING; later updates are ignored (grpc-go semantics)."""
        self._shutdown = True
        for svc in list(self._status):
            self._set(svc, NOT_SERVING)

    def resume(self) -> None:
        self._shutdown = False
        for svc in list(self._status):
            self._set(svc, SERVING)

    async def Check(self, request, context):
        st = self._status.get(request.service)
        if st is None:
            await context.abort(grpc.StatusCode.NOT_FOUND, "unknown service")
        return proto.HealthCheckResponse(status=st)

    async def Watch(self, request, context):
        svc = request.service
        q: asyncio.Queue = asyncio.Queue()
        self._watchers.setdefault(svc, set()).add(q)
        try:
            last = None
            cur = self._status.get(svc, SERVICE_UNKNOWN)
            yield proto.HealthCheckResponse(status=cur)
            last = cur
            while True:
                st = await q.get()
                if st != last:
                    last = st
                    yield proto.HealthCheckResponse(status=st)
        finally:
            self._watchers.get(svc, set()).discard(q)

    def handler(self) -> grpc.GenericRpcHandler:
        return grpc.method_handlers_generic_handler(proto.HEALTH_SERVICE, {
            "Check": grpc.unary_unary_rpc_method_handler(
                self.Check, request_deserializer=proto.HealthCheckRequest.FromString,
                response_serializer=proto.HealthCheckResponse.SerializeToString),
            "Watch": grpc.unary_stream_rpc_method_handler(
                self.Watch, request_deserializer=proto.HealthCheckRequest.FromString,
                response_serializer=proto.HealthCheckResponse.SerializeToString),
        })
