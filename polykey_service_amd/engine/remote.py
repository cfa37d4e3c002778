"""Multi-process request-level data parallelism: one gRPC front end, one engine process per GPU.

SURVEY.md §2.3 "DP": N independent TP=1 engines on N GPUs behind ONE front end whose router
sends each request to the least-loaded engine.  Each engine runs in its own process (its own
GIL, its own HIP device -- one rank per GPU under torchrun) and is reached over a local TCP
socket; rank 0 hosts the front end next to its own engine, which it calls directly.

Wire format: 4-byte little-endian length + a msgpack map per frame.
    front end -> engine   {"op": "add", "rid", "prompt": [ids], "params": {...}, "final": bool}
                          {"op": "abort", "rid"}      {"op": "stop"}
    engine -> front end   {"op": "out", "items": [[rid, new_ids, finished, reason, n_prompt, n_out,
                                                   metrics | null, error | null], ...]}
One "out" frame carries every request's news of one engine step (written by the engine thread
itself, no event loop in between); a request submitted with ``final`` (unary RPCs without stop
strings) is reported once, with all its tokens, when it finishes.
"""
from __future__ import annotations

import asyncio
import dataclasses
import socket
import struct
import threading
import time
import uuid
from typing import Dict, List, Optional, Tuple

import msgpack

from .sequence import RequestOutput, SamplingParams

_HDR = struct.Struct("<I")


def _send(sock: socket.socket, lock: threading.Lock, obj) -> None:
    data = msgpack.packb(obj, use_bin_type=True)
    with lock:
        sock.sendall(_HDR.pack(len(data)) + data)


def _recv_exact(sock: socket.socket, n: int) -> Optional[bytes]:
    buf = bytearray()
    while len(buf) < n:
        chunk = sock.recv(n - len(buf))
        if not chunk:
            return None
        buf += chunk
    return bytes(buf)


def _recv(sock: socket.socket):
    hdr = _recv_exact(sock, _HDR.size)
    if hdr is None:
        return None
    body = _recv_exact(sock, _HDR.unpack(hdr)[0])
    return None if body is None else msgpack.unpackb(body, raw=False)


def _params_dict(p: SamplingParams) -> dict:
    d = dataclasses.asdict(p)
    d["stop_token_ids"] = list(d["stop_token_ids"])
    d["stop"] = list(d["stop"])
    return d


# --------------------------------------------------------------------------- engine side
class EngineServer:
    """Serves one :class:`~polykey_service_amd.engine.async_llm.AsyncLLM` to front ends.

    ``serve(n)`` blocks: it accepts ``n`` authenticated front-end connections (the rank-0 front
    end: 1), feeds their commands to the engine, and returns once every one of them has sent
    "stop" or closed; outputs go back
    from the engine thread through :meth:`AsyncLLM.set_external_sink`, each to the connection
    that submitted the request."""

    def __init__(self, llm, host: str = "127.0.0.1", port: int = 0, token: Optional[str] = None):
        self.llm = llm
        self.lsock = socket.create_server((host, port))
        self.port = self.lsock.getsockname()[1]
        # shared secret the front end must present in its first frame (None: no check)
        self.token = token
        self._lock = threading.Lock()
        self._conns: Dict[int, Tuple[socket.socket, threading.Lock]] = {}
        self._owner: Dict[str, int] = {}   # rid -> connection that submitted it
        self._final: Dict[str, List] = {}  # rid -> tokens so far (final-only requests)

    def _sink(self, items) -> None:
        """Engine thread: one frame per front end with this step's outputs of its requests."""
        per: Dict[int, list] = {}
        with self._lock:
            for rid, o in items:
                cid = self._owner.get(rid)
                if isinstance(o, BaseException):
                    self._final.pop(rid, None)
                    self._owner.pop(rid, None)
                    per.setdefault(cid, []).append([rid, [], True, "error", 0, 0, None, str(o)])
                    continue
                acc = self._final.get(rid)
                if acc is not None:
                    acc.extend(o.new_token_ids)
                    if not o.finished:
                        continue
                    del self._final[rid]
                    ids = acc
                else:
                    ids = o.new_token_ids
                if o.finished:
                    self._owner.pop(rid, None)
                per.setdefault(cid, []).append([rid, list(ids), o.finished, o.finish_reason, o.num_prompt_tokens,
                                                o.num_output_tokens, o.metrics, None])
            conns = {cid: self._conns.get(cid) for cid in per}
        for cid, out in per.items():
            c = conns.get(cid)
            if c is None:
                continue
            try:
                _send(c[0], c[1], {"op": "out", "items": out})
            except OSError:
                pass  # front end gone: its reader sees the closed connection and stops

    def _accept(self) -> socket.socket:
        """The next connection whose hello frame carries the shared token (others are closed)."""
        while True:
            conn, _ = self.lsock.accept()
            if self.token is None:
                return conn
            conn.settimeout(10.0)
            try:
                hello = _recv(conn)
            except (OSError, ValueError, msgpack.exceptions.ExtraData, msgpack.exceptions.UnpackException):
                hello = None
            if isinstance(hello, dict) and hello.get("op") == "hello" and hello.get("token") == self.token:
                conn.settimeout(None)
                return conn
            conn.close()

    def _read(self, cid: int, conn: socket.socket) -> None:
        try:
            while True:
                msg = _recv(conn)
                if msg is None or msg.get("op") == "stop":
                    break
                if msg["op"] == "add":
                    rid = msg["rid"]
                    with self._lock:
                        self._owner[rid] = cid
                        if msg.get("final"):
                            self._final[rid] = []
                    self.llm.submit_external(rid, msg["prompt"], SamplingParams(**msg["params"]))
                elif msg["op"] == "abort":
                    with self._lock:
                        self._final.pop(msg["rid"], None)  # the engine reports nothing more for it
                        self._owner.pop(msg["rid"], None)
                    self.llm.abort_external(msg["rid"])
        except OSError:
            pass
        finally:
            with self._lock:
                self._conns.pop(cid, None)
            try:
                conn.close()
            except OSError:
                pass

    def serve(self, n_clients: int = 1) -> None:
        self.llm.set_external_sink(self._sink)
        readers = []
        try:
            for cid in range(n_clients):
                conn = self._accept()
                conn.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
                with self._lock:
                    self._conns[cid] = (conn, threading.Lock())
                t = threading.Thread(target=self._read, args=(cid, conn), name=f"polykey-engine-srv-{cid}",
                                     daemon=True)
                t.start()
                readers.append(t)
            for t in readers:
                t.join()
        finally:
            self.llm.set_external_sink(None)
            self.lsock.close()


# ---------------------------------------------------------------------------- front end
class RemoteEngine:
    """Front-end handle of an engine in another process; duck-types ``AsyncLLM`` for the
    router (:class:`~polykey_service_amd.adapters.local_llm.ReplicaPool`) and the tools."""

    def __init__(self, addr: Tuple[str, int], tokenizer, name: str = "remote", connect_timeout: float = 120.0,
                 token: Optional[str] = None):
        self.tokenizer = tokenizer
        self.name = name
        self.on_fatal = None
        self.watchdog_s = 0.0
        self.dead: Optional[BaseException] = None
        deadline = time.monotonic() + connect_timeout
        while True:
            try:
                self.sock = socket.create_connection(addr, timeout=5.0)
                break
            except OSError:
                if time.monotonic() > deadline:
                    raise
                time.sleep(0.05)
        self.sock.settimeout(None)
        self.sock.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
        self._wlock = threading.Lock()
        if token is not None:
            _send(self.sock, self._wlock, {"op": "hello", "token": token})
        self._lock = threading.Lock()
        self._streams: Dict[str, Tuple[asyncio.AbstractEventLoop, asyncio.Queue]] = {}
        self._closed = False
        self._reader = threading.Thread(target=self._read, name=f"polykey-remote-{name}", daemon=True)
        self._reader.start()

    def load(self) -> int:
        return len(self._streams)

    def healthy(self) -> bool:
        return self.dead is None

    def _read(self) -> None:
        try:
            while True:
                msg = _recv(self.sock)
                if msg is None:
                    break
                if msg.get("op") != "out":
                    continue
                by_loop: Dict[asyncio.AbstractEventLoop, list] = {}
                with self._lock:
                    for rid, ids, fin, reason, npr, nout, metrics, err in msg["items"]:
                        ent = self._streams.get(rid)
                        if ent is None:
                            continue
                        item = RuntimeError(err) if err else RequestOutput(rid, ids, fin, reason, npr, nout, metrics)
                        by_loop.setdefault(ent[0], []).append((ent[1], item))
                for loop, batch in by_loop.items():
                    try:
                        loop.call_soon_threadsafe(_fanout, batch)
                    except RuntimeError:
                        pass
        except OSError as e:
            if not self._closed:
                self.dead = e
        finally:
            if not self._closed and self.dead is None:
                self.dead = ConnectionError(f"engine {self.name} closed the connection")
            if self.dead is not None:
                with self._lock:
                    ents = list(self._streams.values())
                for loop, q in ents:
                    try:
                        loop.call_soon_threadsafe(q.put_nowait, RuntimeError(f"engine {self.name} is dead"))
                    except RuntimeError:
                        pass
                if self.on_fatal is not None:
                    try:
                        self.on_fatal(self.dead)
                    except Exception:
                        pass

    async def generate(self, prompt_ids: List[int], params: SamplingParams, request_id: Optional[str] = None,
                       final_only: bool = False):
        if self.dead is not None:
            raise RuntimeError(f"engine {self.name} is dead: {self.dead}")
        rid = request_id or uuid.uuid4().hex
        q: asyncio.Queue = asyncio.Queue()
        with self._lock:
            if rid in self._streams:
                raise ValueError(f"duplicate request id {rid}")
            self._streams[rid] = (asyncio.get_running_loop(), q)
        finished = False
        try:
            _send(self.sock, self._wlock, {"op": "add", "rid": rid, "prompt": list(prompt_ids),
                                           "params": _params_dict(params), "final": bool(final_only)})
            while True:
                item = await q.get()
                if isinstance(item, BaseException):
                    finished = True
                    raise item
                yield item
                if item.finished:
                    finished = True
                    return
        finally:
            with self._lock:
                self._streams.pop(rid, None)
            if not finished and self.dead is None:
                try:
                    _send(self.sock, self._wlock, {"op": "abort", "rid": rid})
                except OSError:
                    pass

    async def generate_all(self, prompt_ids: List[int], params: SamplingParams, request_id: Optional[str] = None):
        toks: List[int] = []
        last = None
        async for out in self.generate(prompt_ids, params, request_id, final_only=True):
            toks.extend(out.new_token_ids)
            last = out
        return toks, last

    def shutdown(self, timeout: Optional[float] = None) -> None:
        if self._closed:
            return
        self._closed = True
        try:
            _send(self.sock, self._wlock, {"op": "stop"})
        except OSError:
            pass
        try:
            self.sock.shutdown(socket.SHUT_RDWR)
        except OSError:
            pass
        self.sock.close()
        self._reader.join(timeout or 10.0)

    async def aclose(self) -> None:
        await asyncio.get_running_loop().run_in_executor(None, self.shutdown)


def dp_gateway(llm, st, group=None):
    """Wire the DP ranks (tp = 1, one engine per rank) to ONE gRPC front end on rank 0.

    Collective over ``group`` (default: the world): every rank but 0 serves its ``llm`` to rank 0
    and blocks until the front end stops it (returns None); rank 0 returns a
    :class:`~polykey_service_amd.adapters.local_llm.ReplicaPool` over its own ``llm`` and a
    :class:`RemoteEngine` per other rank (least-loaded routing).

    (Round 4 retired the SO_REUSEPORT variant -- one address, an acceptor per rank over a
    shared-memory load board: it cost 1.8-2.4 % against per-rank endpoints when it ran clean and
    stalled intermittently on the shared-GPU rehearsal, profiles/r3_gateway_ab.txt.  Per-rank
    endpoints (bench.py's replicas, one gRPC server per GPU behind any TCP load balancer) are the
    DP design; this single front end serves deployments that need one address.)"""
    import os
    import secrets

    import torch.distributed as dist

    from ..adapters.local_llm import ReplicaPool
    # one node: loopback only; several nodes: every rank listens on all interfaces and
    # advertises its host name (POLYKEY_GATEWAY_HOST overrides what it advertises)
    single_node = int(os.environ.get("LOCAL_WORLD_SIZE", str(st.world_size))) == st.world_size
    bind = "127.0.0.1" if single_node else "0.0.0.0"
    advertise = os.environ.get("POLYKEY_GATEWAY_HOST") or ("127.0.0.1" if single_node else socket.gethostname())
    # rank 0 draws the shared token; every engine server accepts only a front end that presents it
    tok = [secrets.token_hex(16) if st.rank == 0 else None]
    dist.broadcast_object_list(tok, src=0, group=group)
    server = EngineServer(llm, host=bind, token=tok[0]) if st.rank != 0 else None
    addrs: List = [None] * st.world_size
    dist.all_gather_object(addrs, (advertise, server.port) if server is not None else None, group=group)
    if server is not None:
        server.serve()
        return None
    remotes = [RemoteEngine(tuple(addrs[r]), llm.tokenizer, name=f"rank{r}", token=tok[0])
               for r in range(1, st.world_size)]
    return ReplicaPool([llm] + remotes)


def _fanout(batch) -> None:
    for q, item in batch:
        q.put_nowait(item)
