"""Async face of the engine: the continuous-batching loop runs on its own thread; gRPC
handlers on the asyncio loop submit requests and consume per-request token streams.

Thread → loop hand-off is batched: one ``call_soon_threadsafe`` per engine step delivers
every request's new tokens (64 streams × 1 token each would otherwise be 64 self-pipe
wake-ups per step).  A request whose consumer goes away (client cancelled / disconnected)
is aborted on the engine thread, which frees its KV blocks.  If the engine
loop dies, every open stream receives the error and ``on_fatal`` fires (the server flips
health to NOT_SERVING).
"""
from __future__ import annotations

import asyncio
import collections
import contextlib
import gc
import os
import sys
import threading
import time
import traceback
import uuid
from typing import AsyncIterator, Callable, Deque, Dict, List, Optional, Tuple

from .llm_engine import LLMEngine
from .sequence import RequestOutput, SamplingParams


class EngineDeadError(RuntimeError):
    pass


def bind_device(dev) -> None:
    """Make ``dev`` the calling thread's current HIP device (no-op for CPU / None)."""
    if dev is not None and getattr(dev, "type", None) == "cuda":
        import torch
        torch.cuda.set_device(dev)


@contextlib.contextmanager
def device_guard(dev):
    """``torch.cuda.device(dev)`` for a CUDA ``dev``, nothing otherwise: build an engine on a GPU
    other than the thread's current one (its native launches go to the current device)."""
    if dev is not None and getattr(dev, "type", None) == "cuda":
        import torch
        with torch.cuda.device(dev):
            yield
    else:
        yield


class AsyncLLM:
    def __init__(self, engine: LLMEngine, on_fatal: Optional[Callable[[BaseException], None]] = None,
                 watchdog_s: float = 0.0, metrics=None):
        from ..utils import metrics as _m
        self.engine = engine
        # pipelined steps: RequestOutputs are built / delivered while the GPU runs the next step
        engine.overlap = os.environ.get("POLYKEY_OVERLAP_STEPS", "1") == "1"
        self.metrics = metrics if metrics is not None else _m.current()
        self.tokenizer = engine.tokenizer
        self.on_fatal = on_fatal
        self._cmds: Deque[Tuple[str, object]] = collections.deque()
        self._wake = threading.Event()
        self._streams: Dict[str, Tuple[asyncio.AbstractEventLoop, asyncio.Queue]] = {}
        # requests submitted by another process's front end (engine/remote.py EngineServer):
        # their outputs go to the external sink, called on the engine thread once per step
        self._external: set = set()
        self._external_sink: Optional[Callable[[list], None]] = None
        self._lock = threading.Lock()
        self._stop = False
        self.dead: Optional[BaseException] = None
        self.last_step_time = time.monotonic()
        # monotonic start of the step in flight (None between steps): the watchdog only judges a
        # step that has started and not returned, never an idle gap before a new request
        self.step_started: Optional[float] = None
        self.watchdog_s = watchdog_s
        self.stats = {"steps": 0, "requests": 0, "output_tokens": 0, "step_time_s": 0.0, "arrival_waits": 0}
        # Arrival coalescing: an idle engine that receives a request keeps collecting arrivals
        # for up to ARRIVAL_WINDOW_MS (while they keep coming at most ARRIVAL_GAP_MS apart) until
        # one prefill step is full.  A burst of requests -- closed-loop clients re-submitting
        # together -- is then prefilled in full budget-sized steps instead of a first step holding
        # only the earliest few (8B bench wave: prefill 45 + 87 + 100 ms -> 2 full steps).  A lone
        # request waits one gap.  0 disables.
        self.arrival_window_s = float(os.environ.get("POLYKEY_ARRIVAL_WINDOW_MS", "8")) / 1e3
        self.arrival_gap_s = float(os.environ.get("POLYKEY_ARRIVAL_GAP_MS", "2")) / 1e3

        # The engine thread and the asyncio (gRPC) thread share the GIL.  CPython's default 5 ms
        # switch interval lets a burst of RPC handling hold the engine thread off for whole
        # decode steps (the GPU idles meanwhile); a short interval hands the GIL over promptly.
        sys.setswitchinterval(float(os.environ.get("POLYKEY_SWITCH_INTERVAL_MS", "2")) / 1e3)
        # Collector pauses: the engine, its weights' Python wrappers and the captured graphs are
        # long-lived -- gc.freeze() moves them out of every later collection, and a larger
        # generation-0 threshold keeps the per-step garbage (outputs, RPC messages) from
        # triggering collections mid-wave.  A full collection of the serving heap stalled a bench
        # wave by ~50 ms (profiles/r6_gc.md).  POLYKEY_GC_FREEZE=0 keeps CPython's defaults.
        if os.environ.get("POLYKEY_GC_FREEZE", "1") != "0":
            gc.collect()
            gc.freeze()
            gc.set_threshold(50000, 20, 100)
        self._fatal_sent = False
        if os.environ.get("POLYKEY_DRAIN_BEFORE_SCHEDULE", "1") != "0":
            engine.before_schedule = self._drain_cmds
        self._thread = threading.Thread(target=self._run, name="polykey-engine", daemon=True)
        self._thread.start()
        self._watchdog = threading.Thread(target=self._watch, name="polykey-watchdog", daemon=True)
        self._watchdog.start()

    # ---------------------------------------------------------------- client side
    def load(self) -> int:
        """Unfinished + queued requests (the DP router's least-loaded metric)."""
        return self.engine.scheduler.num_unfinished() + len(self._cmds)

    # ---------------------------------------------------------- remote front end
    def set_external_sink(self, sink: Optional[Callable[[list], None]]) -> None:
        self._external_sink = sink

    def submit_external(self, rid: str, prompt_ids: List[int], params: SamplingParams) -> None:
        if self.dead is not None:
            sink = self._external_sink
            if sink is not None:
                sink([(rid, EngineDeadError(f"engine is dead: {self.dead}"))])
            return
        with self._lock:
            self._external.add(rid)
            self._cmds.append(("add", (rid, prompt_ids, params)))
        self._wake.set()

    def abort_external(self, rid: str) -> None:
        with self._lock:
            if rid not in self._external:
                return
            self._external.discard(rid)
            self._cmds.append(("abort", rid))
        self._wake.set()

    async def generate(self, prompt_ids: List[int], params: SamplingParams,
                       request_id: Optional[str] = None, final_only: bool = False) -> AsyncIterator[RequestOutput]:
        if self.dead is not None:
            raise EngineDeadError(f"engine is dead: {self.dead}")
        rid = request_id or uuid.uuid4().hex
        loop = asyncio.get_running_loop()
        q: asyncio.Queue = asyncio.Queue()
        with self._lock:
            if rid in self._streams:
                raise ValueError(f"duplicate request id {rid}")
            self._streams[rid] = (loop, q)
            self._cmds.append(("add", (rid, prompt_ids, params)))
        self._wake.set()
        finished = False
        try:
            while True:
                item = await q.get()
                # coalesce whatever else already arrived: a lagging consumer gets one message
                # carrying several tokens instead of one message per engine step
                while not isinstance(item, BaseException) and not item.finished and not q.empty():
                    nxt = q.get_nowait()
                    if isinstance(nxt, BaseException):
                        item = nxt
                        break
                    item = RequestOutput(item.request_id, item.new_token_ids + nxt.new_token_ids, nxt.finished,
                                         nxt.finish_reason, nxt.num_prompt_tokens, nxt.num_output_tokens,
                                         nxt.metrics)
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
                if not finished:
                    self._cmds.append(("abort", rid))
            if not finished:
                self._wake.set()

    async def generate_all(self, prompt_ids: List[int], params: SamplingParams,
                           request_id: Optional[str] = None) -> Tuple[List[int], RequestOutput]:
        toks: List[int] = []
        last = None
        async for out in self.generate(prompt_ids, params, request_id):
            toks.extend(out.new_token_ids)
            last = out
        return toks, last

    def shutdown(self, timeout: Optional[float] = None) -> None:
        """Stop the engine thread (DP attention + EP: waits until every rank has asked to stop,
        up to ``timeout``; default 10 s, 600 s in lockstep)."""
        if timeout is None:
            timeout = 600.0 if self.engine.lockstep else 10.0
        self._stop = True
        self._wake.set()
        self._thread.join(timeout)
        if self._watchdog is not threading.current_thread():
            self._watchdog.join(2.0)  # sleeps <= 1 s between checks; not left running into exit
        try:
            self.engine.shutdown()
        except Exception:
            pass

    async def aclose(self) -> None:
        await asyncio.get_running_loop().run_in_executor(None, self.shutdown)

    def stalled_for(self) -> float:
        """Seconds the step in flight has been running (0 between steps)."""
        t0 = self.step_started
        return 0.0 if t0 is None else time.monotonic() - t0

    def _watch(self) -> None:
        """Step watchdog: a step in flight for ``watchdog_s`` (a collective hung
        on a dead peer, a wedged GPU) kills the engine: its communicators
        are aborted (the hung RCCL call returns, IPC collectives stop waiting), every stream
        gets the error and ``on_fatal`` fires -- the server goes NOT_SERVING and exits non-zero
        for its supervisor to restart the group.  Disabled while ``watchdog_s`` is 0."""
        while not self._stop and self.dead is None:
            time.sleep(0.5 if self.watchdog_s else 1.0)
            w = self.watchdog_s
            if not w or self.dead is not None or self._stop:
                continue
            if self.stalled_for() > w:
                err = TimeoutError(f"engine step stalled for more than {w:.0f} s (hung collective or GPU)")
                self.dead = err
                try:
                    self.engine.runner.abort_comms()
                except Exception:  # noqa: BLE001
                    pass
                with self._lock:
                    rids = list(self._streams) + list(self._external)
                self._deliver([(r, EngineDeadError(f"engine stalled: {err}")) for r in rids])
                self._fatal(err)

    def _fatal(self, e: BaseException) -> None:
        if self._fatal_sent:
            return
        self._fatal_sent = True
        if self.on_fatal is not None:
            try:
                self.on_fatal(e)
            except Exception:
                pass

    def healthy(self) -> bool:
        if self.dead is not None:
            return False
        if self.watchdog_s:
            return self.stalled_for() < self.watchdog_s
        return True

    # ---------------------------------------------------------------- engine side
    def _drain_cmds(self) -> None:
        with self._lock:
            cmds = list(self._cmds)
            self._cmds.clear()
        for kind, arg in cmds:
            if kind == "add":
                rid, prompt, params = arg
                try:
                    self.engine.add_request(prompt, params, rid)
                    self.stats["requests"] += 1
                except Exception as e:  # noqa: BLE001 - reported to that request only
                    self._deliver([(rid, ValueError(str(e)))])
            elif kind == "abort":
                self.engine.abort(arg)

    def _coalesce_arrivals(self) -> None:
        eng = self.engine
        deadline = time.monotonic() + self.arrival_window_s
        self.stats["arrival_waits"] += 1
        while not self._stop and eng.first_step_unfilled():
            left = deadline - time.monotonic()
            if left <= 0:
                return
            with self._lock:
                pending = bool(self._cmds)
                if not pending:
                    self._wake.clear()
            if not pending and not self._wake.wait(min(self.arrival_gap_s, left)):
                return  # the burst is over
            self._drain_cmds()

    def _deliver(self, items) -> None:
        by_loop: Dict[asyncio.AbstractEventLoop, list] = {}
        external = []
        with self._lock:
            for rid, item in items:
                if rid in self._external:
                    external.append((rid, item))
                    if isinstance(item, BaseException) or item.finished:
                        self._external.discard(rid)
                    continue
                ent = self._streams.get(rid)
                if ent is not None:
                    by_loop.setdefault(ent[0], []).append((ent[1], item))
        sink = self._external_sink
        if external and sink is not None:
            sink(external)
        for loop, batch in by_loop.items():
            try:
                loop.call_soon_threadsafe(_fanout, batch)
            except RuntimeError:
                pass  # loop closed

    def _profiler(self):
        """``POLYKEY_TORCH_PROFILE=<dir>``: torch.profiler over engine steps (skip 20, warm up 5,
        record 20), exported as a Chrome trace into <dir>."""
        out = os.environ.get("POLYKEY_TORCH_PROFILE")
        if not out:
            return None
        import torch
        from torch.profiler import ProfilerActivity, profile, schedule, tensorboard_trace_handler
        acts = [ProfilerActivity.CPU] + ([ProfilerActivity.CUDA] if torch.cuda.is_available() else [])
        prof = profile(activities=acts, schedule=schedule(wait=20, warmup=5, active=20, repeat=1),
                       on_trace_ready=tensorboard_trace_handler(out))
        prof.start()
        return prof

    def _run(self) -> None:
        eng = self.engine
        # the HIP device is per thread: every native launch of this engine (ops/native.py, current
        # stream of the current device) must target the engine's GPU, not cuda:0 (several
        # engines of one process on different GPUs: attach_models / ReplicaPool)
        bind_device(getattr(eng, "device", None))
        prof = self._profiler()
        try:
            while True:
                self._drain_cmds()
                if eng.lockstep:
                    # DP attention + EP: one vote per iteration on every rank; the loop ends only
                    # when every rank is stopping and none has work left (a rank leaving alone
                    # would strand the others in their next all-to-all)
                    busy, all_stop = eng.lockstep_vote(self._stop)
                    if all_stop and not busy:
                        break
                else:
                    if self._stop:
                        break
                    busy = eng.has_unfinished()
                if not busy:
                    self._wake.wait(0.05)
                    self._wake.clear()
                    continue
                if not eng.lockstep and self.arrival_window_s > 0 and eng.idle_with_waiting():
                    self._coalesce_arrivals()
                t0 = time.perf_counter()
                self.step_started = time.monotonic()
                outs = eng.step()
                self.step_started = None
                if prof is not None:
                    prof.step()
                dt = time.perf_counter() - t0
                self.stats["step_time_s"] += dt
                if self.metrics is not None:
                    self.metrics.observe_step(eng, dt, outs)
                self.stats["steps"] += 1
                self.last_step_time = time.monotonic()
                if outs:
                    self.stats["output_tokens"] += sum(len(o.new_token_ids) for o in outs)
                    self._deliver([(o.request_id, o) for o in outs])
        except BaseException as e:  # noqa: BLE001
            if self.dead is None:
                self.dead = e
            traceback.print_exc()
            try:  # a peer failed: let collectives of this rank stop waiting on it
                eng.runner.abort_comms()
            except Exception:  # noqa: BLE001
                pass
            with self._lock:
                rids = list(self._streams) + list(self._external)
            self._deliver([(r, EngineDeadError(f"engine loop failed: {e!r}")) for r in rids])
            self._fatal(e)
        finally:
            if prof is not None:
                prof.stop()


def _fanout(batch) -> None:
    for q, item in batch:
        q.put_nowait(item)
