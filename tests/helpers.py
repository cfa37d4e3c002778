"""Shared test helpers."""
import asyncio
import io
import json
import threading

from polykey_service_amd.server import PolykeyServer
from polykey_service_amd.service import ToolRouter
from polykey_service_amd.utils import slog


class ServerThread:
    """Runs a PolykeyServer on its own event loop thread."""

    def __init__(self, service=None, **server_kw):
        self.server_kw = server_kw
        self.log = io.StringIO()
        self.service = service or ToolRouter()
        self.loop = asyncio.new_event_loop()
        self.ready = threading.Event()
        self.t = threading.Thread(target=self._run, daemon=True)

    def _run(self):
        asyncio.set_event_loop(self.loop)
        self.srv = PolykeyServer(self.service, slog.Logger(self.log), "127.0.0.1:0", own_service=False,
                                 **self.server_kw)
        self.port = self.loop.run_until_complete(self.srv.start())
        self.ready.set()
        self.loop.run_forever()

    def __enter__(self):
        self.t.start()
        self.ready.wait(10)
        self.addr = f"127.0.0.1:{self.port}"
        return self

    def stop(self, grace=1.0):
        fut = asyncio.run_coroutine_threadsafe(self.srv.stop(grace), self.loop)
        fut.result(10)

    def __exit__(self, *a):
        if not self.srv._stopped.is_set():
            self.stop()
        self.loop.call_soon_threadsafe(self.loop.stop)
        self.t.join(5)

    def records(self, settle=0.2):
        import time
        time.sleep(settle)  # the "finished" line is written after the response is sent
        return [json.loads(l) for l in self.log.getvalue().splitlines() if l.strip()]


