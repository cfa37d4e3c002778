"""L1 transport / process entry (reference ``cmd/polykey/main.go:54-121``).

Startup sequence mirrors the reference: JSON logger on stdout → listen on ``LISTEN_ADDR``
(default ``:50051``) → gRPC server with keepalive + logging interceptor → reflection →
health (SERVING for ``polykey.v2.PolykeyService`` and ``""``) → log every registered
service and method → ``"server starting" {address}`` → wait for SIGINT/SIGTERM →
``"server shutting down"`` → health NOT_SERVING → graceful stop → ``"server stopped"``.

Transport parameters (``main.go:68-72``): MaxConnectionIdle 5 min, Time 2 h, Timeout 20 s.
[NEW] a keepalive *enforcement* policy (min ping interval 5 s, pings allowed without
streams): the reference's clients ping every 10 s with PermitWithoutStream while its server
keeps grpc-go's 5 min default, which ends long-lived connections with GOAWAY
``too_many_pings``.
[NEW] optional TLS: with a PEM certificate chain and key the port is bound
with ``grpc.ssl_server_credentials`` instead of the reference's insecure transport.
"""
from __future__ import annotations

import asyncio
import signal
from typing import List, Optional

import grpc

from .. import proto
from ..utils import slog
from .health import SERVING, HealthServicer
from .interceptors import LoggingInterceptor
from .reflection import ReflectionServicer
from .rpc import SERVICE_METHODS, PolykeyServicer

MIB = 1024 * 1024

SERVER_OPTIONS = [
    ("grpc.max_connection_idle_ms", 5 * 60 * 1000),
    ("grpc.keepalive_time_ms", 2 * 3600 * 1000),
    ("grpc.keepalive_timeout_ms", 20 * 1000),
    ("grpc.keepalive_permit_without_calls", 1),
    ("grpc.http2.min_recv_ping_interval_without_data_ms", 5 * 1000),
    ("grpc.http2.max_ping_strikes", 0),
    ("grpc.max_receive_message_length", 4 * MIB),
    ("grpc.max_send_message_length", 64 * MIB),
]


def grpc_bind_address(addr: str) -> str:
    """Go ``net.Listen`` style ``":50051"`` → ``"[::]:50051"``."""
    if addr.startswith(":"):
        return "[::]" + addr
    return addr


class PolykeyServer:
    def __init__(self, service, logger: Optional[slog.Logger] = None, listen_addr: str = ":50051",
                 metrics=None, extra_handlers: Optional[List] = None, own_service: bool = True,
                 tls_cert: str = "", tls_key: str = ""):
        self.logger = logger or slog.Logger()
        self.tls = (tls_cert, tls_key) if tls_cert and tls_key else None
        self.listen_addr = listen_addr
        self.service = service
        self.health = HealthServicer()
        self.metrics = metrics
        observer = metrics.observe_rpc if metrics is not None else None
        self.server = grpc.aio.server(interceptors=[LoggingInterceptor(self.logger, observer)],
                                      options=SERVER_OPTIONS)
        self.port: Optional[int] = None
        self._extra = extra_handlers or []
        self.own_service = own_service  # stop() also closes the service (engine thread)
        self._stopped = asyncio.Event()
        self._quit: Optional[asyncio.Event] = None
        # the engine loop died (HIP error, TP peer timeout, ...): health goes NOT_SERVING at once
        # and, with exit_on_fatal, the process stops with a non-zero status for its supervisor
        # (compose ``restart: unless-stopped``, Kubernetes) to restart it
        self.fatal_error: Optional[BaseException] = None
        self.exit_on_fatal = True
        self.fatal_grace_s = 2.0

    async def start(self) -> int:
        bind = grpc_bind_address(self.listen_addr)
        try:
            if self.tls is not None:
                with open(self.tls[0], "rb") as f:
                    chain = f.read()
                with open(self.tls[1], "rb") as f:
                    key = f.read()
                self.port = self.server.add_secure_port(bind, grpc.ssl_server_credentials([(key, chain)]))
            else:
                self.port = self.server.add_insecure_port(bind)
        except RuntimeError as e:
            self.logger.error("failed to listen", error=str(e))
            raise
        refl = [ReflectionServicer(SERVICE_METHODS.keys(), v) for v in ("v1alpha", "v1")]
        handlers = [PolykeyServicer(self.service, self.logger).handler(), self.health.handler()]
        handlers += [r.handler() for r in refl] + self._extra
        self.server.add_generic_rpc_handlers(handlers)
        self.health.set_serving_status(proto.POLYKEY_SERVICE, SERVING)
        self.health.set_serving_status("", SERVING)

        self.logger.info("Registered services:")
        for name, methods in SERVICE_METHODS.items():
            self.logger.info("Service registered", name=name, methods=len(methods))
            for m in methods:
                self.logger.info("Method available", service=name, method=m)

        extra = {"tls": True} if self.tls is not None else {}  # the reference's schema otherwise
        self.logger.info("server starting", address=self.listen_addr, **extra)
        await self.server.start()
        return self.port

    async def stop(self, grace: float = 10.0) -> None:
        self.logger.info("server shutting down")
        w = getattr(self, "_watch", None)
        if w is not None:
            w.cancel()
        self.health.shutdown()
        await self.server.stop(grace)
        close = getattr(self.service, "aclose", None) if self.own_service else None
        if close is not None:
            await close()
        self.logger.info("server stopped")
        self._stopped.set()

    def watch_backend(self, llm, interval: float = 1.0) -> "asyncio.Task":
        """Failure detection: the health status follows the engine — NOT_SERVING
        as soon as its loop dies (``on_fatal``) or its watchdog says a step has stalled."""
        from .health import NOT_SERVING
        loop = asyncio.get_running_loop()

        def fatal(exc):
            self.logger.error("engine loop died", error=repr(exc))
            self.fatal_error = exc
            loop.call_soon_threadsafe(self.health.set_serving_status, proto.POLYKEY_SERVICE, NOT_SERVING)
            loop.call_soon_threadsafe(self.health.set_serving_status, "", NOT_SERVING)
            if self.exit_on_fatal:
                # give probes a moment to observe NOT_SERVING, then leave serve_until_signal
                loop.call_soon_threadsafe(loop.call_later, self.fatal_grace_s, self._request_quit)

        llm.on_fatal = fatal

        async def poll():
            while True:
                await asyncio.sleep(interval)
                ok = llm.healthy()
                st = SERVING if ok else NOT_SERVING
                if self.health.get(proto.POLYKEY_SERVICE) != st:
                    self.logger.warn("backend health changed", serving=ok)
                    self.health.set_serving_status(proto.POLYKEY_SERVICE, st)
                    self.health.set_serving_status("", st)

        self._watch = asyncio.create_task(poll())
        return self._watch

    def _request_quit(self) -> None:
        if self._quit is not None:
            self._quit.set()

    async def serve_until_signal(self, grace: float = 10.0) -> int:
        """Serve until SIGINT/SIGTERM (exit status 0) or a fatal engine failure (status 1)."""
        loop = asyncio.get_running_loop()
        self._quit = quit_ev = asyncio.Event()
        if self.fatal_error is not None and self.exit_on_fatal:
            quit_ev.set()
        for sig in (signal.SIGINT, signal.SIGTERM):
            try:
                loop.add_signal_handler(sig, quit_ev.set)
            except (NotImplementedError, RuntimeError):
                pass
        await quit_ev.wait()
        await self.stop(grace)
        return 1 if self.fatal_error is not None else 0


def build_service(cfg, logger: slog.Logger):
    """Mock router, or router + on-node LLM backend (``cfg.backend == "local"``); None on the ranks
    of a multi-model torchrun job that are not its front end (after they have been stopped)."""
    from ..service.router import ToolRouter
    from ..adapters.security.secret_store import SecretStore

    router = ToolRouter(secret_store=SecretStore.from_env())
    if cfg.backend == "local" and getattr(cfg, "serve_models", ""):
        import os
        if int(os.environ.get("WORLD_SIZE", "1")) > 1:
            # one process per GPU: every model on TP groups of its own, rank 0 the front end; the
            # other ranks return here once the front end has stopped them (no server of their own)
            from ..adapters.local_llm import attach_model_groups
            if attach_model_groups(router, cfg, logger) is None:
                return None
        else:
            from ..adapters.local_llm import attach_models  # several models, one front end
            attach_models(router, cfg, logger)
    elif cfg.backend == "local":
        from ..adapters.local_llm import attach_local_llm
        attach_local_llm(router, cfg, logger)
    elif cfg.backend != "mock":
        raise ValueError(f"unknown backend {cfg.backend!r} (mock|local)")
    return router


async def amain(argv=None) -> int:
    from ..config.server_config import load_server_config

    cfg = load_server_config(argv)
    logger = slog.Logger(level=slog.level_from_name(cfg.log_level))
    slog.set_default(logger)
    metrics = None
    if cfg.metrics_addr:
        from ..utils.metrics import Metrics
        metrics = Metrics.start(cfg.metrics_addr)
    service = build_service(cfg, logger)
    if service is None:  # a model-group rank other than the front end: its engine has been stopped
        return 0
    srv = PolykeyServer(service, logger, cfg.listen_addr, metrics=metrics, tls_cert=cfg.tls_cert,
                        tls_key=cfg.tls_key)
    await srv.start()
    if getattr(service, "llm", None) is not None:
        import os
        service.llm.watchdog_s = float(os.environ.get("POLYKEY_WATCHDOG_S", "60"))
        srv.watch_backend(service.llm)
    http = None
    if cfg.http_addr:
        from ..api.openai import serve_openai
        http = await serve_openai(service, cfg.http_addr, logger)
    rc = await srv.serve_until_signal(cfg.shutdown_grace)
    if http is not None:
        await http.shutdown()
    if rc:
        logger.error("exiting after engine failure", error=repr(srv.fatal_error))
        hard_exit(rc)
    return rc


def hard_exit(rc: int) -> None:
    """Leave NOW with ``rc``: after an engine failure the GPU runtime may still hold a kernel
    that waits on a dead peer, and the interpreter's normal teardown (device sync, process-group
    destruction) would block on it; the supervisor restarts the process (compose
    ``restart: unless-stopped``).  Not an exec: the process just ends."""
    import os
    import sys
    try:
        sys.stdout.flush()
        sys.stderr.flush()
    finally:
        os._exit(rc)


def main(argv=None) -> int:
    return asyncio.run(amain(argv))


if __name__ == "__main__":
    raise SystemExit(main())
