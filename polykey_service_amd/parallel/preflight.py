"""Multi-GPU preflight (SURVEY.md §5.8 "comm backend"): before the first
step, every device collective the engine will use is run once on a few KB of rank-seeded data and
checked against the exact result, which every rank computes locally from the same seeds:

* the direct RCCL communicators (``parallel/rccl.py``): all-reduce, all-gather, reduce-scatter
  (TP / SP), all-to-allv (expert dispatch);
* the IPC collectives of ``csrc/comm/custom_allreduce.hip`` beyond its own start-up all-reduce
  self-test: the one-shot all-gather (LM-head logits) and the fused decode collective
  (``reduce_residual``: partial sum + xGMI peer sum + residual add + norm parts);
* the IPC expert all-to-all (``csrc/comm/ep_alltoall.hip``): dispatch and return.

The verdict of each check is agreed over the group's gloo control group (all ranks keep a path
or none does, so no rank ever waits in a collective its peers abandoned) and a failed path is
disabled -- the engine falls back to the next one (RCCL direct -> torch.distributed, IPC ->
RCCL) exactly as if it had never been created.  One JSON line per rank that saw a failure (and
always on rank 0) records the peer-access matrix, every check and every fallback, so the first
one-rank-per-GPU run on a new node is diagnosable from its log alone.
"""
from __future__ import annotations

import json
import os
import sys
import threading
import time
from typing import Callable, Dict, List, Optional, Tuple

import torch
import torch.distributed as dist

from .state import ParallelState


def _pattern(rank: int, n: int, dtype=torch.bfloat16, device="cpu", salt: int = 0) -> torch.Tensor:
    """Small integers (exact in bf16 and in any summation order) that differ per rank."""
    i = torch.arange(n, dtype=torch.int64)
    return (((i * (rank + 3) + 7 * rank + salt) % 13) - 6).to(dtype).to(device)


def _close(a: torch.Tensor, b: torch.Tensor) -> bool:
    return a.shape == b.shape and bool(torch.equal(a.float().cpu(), b.float().cpu()))


def _sync(dev: torch.device) -> None:
    if dev.type == "cuda":
        torch.cuda.synchronize(dev)


# ----------------------------------------------------------------------------------- checks
def check_rccl(rc, rank: int, world: int, dev: torch.device) -> Dict[str, bool]:
    """all_reduce / all_gather / reduce_scatter / all_to_allv of a direct communicator."""
    out = {}
    n = 1024 * world
    x = _pattern(rank, n, device=dev)
    want = sum(_pattern(r, n) for r in range(world))
    y = rc.all_reduce(x.clone())
    _sync(dev)
    out["all_reduce"] = _close(y, want)
    g = rc.all_gather(_pattern(rank, 256, device=dev, salt=1))
    _sync(dev)
    out["all_gather"] = _close(g, torch.cat([_pattern(r, 256, salt=1) for r in range(world)]))
    rs = rc.reduce_scatter(_pattern(rank, n, device=dev, salt=2))
    _sync(dev)
    full = sum(_pattern(r, n, salt=2) for r in range(world))
    out["reduce_scatter"] = _close(rs, full.view(world, -1)[rank])
    # all-to-allv with uneven splits: rank r sends (r + j) % 3 + 1 rows of width 8 to rank j
    sends = [(rank + j) % 3 + 1 for j in range(world)]
    recvs = [(j + rank) % 3 + 1 for j in range(world)]
    rows = torch.cat([_pattern(rank, sends[j] * 8, device=dev, salt=10 + j).view(-1, 8) for j in range(world)])
    a2a = rc.all_to_allv(rows, recvs, sends)
    _sync(dev)
    out["all_to_allv"] = _close(a2a, torch.cat([_pattern(j, recvs[j] * 8, salt=10 + rank).view(-1, 8)
                                                for j in range(world)]))
    return out


def reduce_residual_widths(world: int) -> List[int]:
    """Residual widths that drive every form of the fused collective: 1024 columns (one-shot for
    W < 4 and for W > 4, whose two-shot needs 256 W-column chunk groups) and the smallest
    multiple of 1024 that holds 256 W columns (two-shot from W = 4; 2048 at W = 8 -- the form a
    70B TP=8 decode step takes)."""
    two = -(-256 * world // 1024) * 1024
    return [1024] if two == 1024 else [1024, two]


def check_custom_ar(car, rank: int, world: int, dev: torch.device) -> Dict[str, bool]:
    """The IPC all-gather and the fused decode collective (reduce_residual, one-shot and two-shot
    forms: parts per 1024 / 256 columns, sized by ``car.nparts``) of custom_ar."""
    out = {}
    x = _pattern(rank, 4 * 64, device=dev, salt=3).view(4, 64)
    if car.supports_gather(x):
        g = car.all_gather_last(x)
        _sync(dev)
        out["all_gather_1shot"] = _close(g, torch.cat([_pattern(r, 256, salt=3).view(4, 64) for r in range(world)], -1))
    M = 2
    # two rounds with different data: every slot parity is reused, so a read served from a stale
    # copy of the previous call's slot (the collectives use no fences: system-scope slot accesses)
    # shows up as a mismatch
    for rnd in range(2):
        for N in reduce_residual_widths(world):
            if not car.supports_reduce_residual(M, N):
                continue
            nparts = car.nparts(M, N)
            part = _pattern(rank, M * N, device=dev, salt=4 + 10 * rnd).view(M, N)
            res0 = _pattern(0, M * N, salt=5 + 10 * rnd).view(M, N)
            residual = res0.to(dev).clone()
            parts = torch.zeros(nparts * M, dtype=torch.float32, device=dev)
            p = car.reduce_residual(part.contiguous(), residual, parts)
            _sync(dev)
            want = res0.float() + sum(_pattern(r, M * N, salt=4 + 10 * rnd).view(M, N).float() for r in range(world))
            want_parts = want.view(M, nparts, N // nparts).pow(2).sum(-1).t()
            form = "2shot" if N // nparts == 256 else "1shot"
            key = f"reduce_residual_{form}_{N}"
            out[key] = out.get(key, True) and _close(residual, want.to(torch.bfloat16)) and tuple(p.shape) == (
                nparts, M) and bool(torch.allclose(p.float().cpu(), want_parts, rtol=1e-5))
    return out


class _Slabs:
    """A split-K slab operand of the fused collective (the fields custom_ar reads of a
    ``gemm.Partial``): ``buf`` fp32 [S * M * N]."""

    def __init__(self, buf: torch.Tensor, S: int, M: int, N: int):
        self.buf, self.S, self.M, self.N = buf, S, M, N

    def view(self) -> torch.Tensor:
        return self.buf[: self.S * self.M * self.N].view(self.S, self.M, self.N)


SERVING_CALLS = 16


def _serving_operands(rank: int, M: int, N: int, calls: int, dev: torch.device):
    """Rank-seeded operands of ``calls`` fused collectives at [M, N]: even calls a bf16 partial,
    odd calls 2 fp32 split-K slabs (p + 0.5, -0.5: the real decode chain's form).  Small integers:
    every sum and every norm part is exact in any order, so a stale or torn slot read cannot hide."""
    ops = []
    for k in range(calls):
        p = _pattern(rank, M * N, dtype=torch.float32, salt=100 + k).view(M, N)
        if k % 2 == 0:
            ops.append(p.to(torch.bfloat16).to(dev).contiguous())
        else:
            buf = torch.cat([(p + 0.5).reshape(-1), torch.full((M * N,), -0.5)]).to(dev)
            ops.append(_Slabs(buf, 2, M, N))
    return ops


def check_custom_ar_serving(car, rank: int, world: int, dev: torch.device, M: int, N: int,
                            calls: int = SERVING_CALLS, graph: Optional[bool] = None) -> Dict[str, object]:
    """The fused decode collective at serving shape: ``calls`` back-to-back
    ``reduce_residual`` calls at [M, N] (M = the largest decode graph bucket, N = hidden) with no
    host synchronisation between them -- every slot parity is reused calls / 2 times while peers
    run up to one call ahead, the window in which a read served from a stale or not-yet-visible
    peer slot shows -- first eagerly, then (on the GPU) captured in a HIP graph and replayed, each
    result compared bit for bit with the locally computed sum.  The timed replay gives the
    per-call time (``collective_us``).  Returns the check dict (booleans) plus that time."""
    graph = dev.type == "cuda" if graph is None else graph
    if not car.supports_reduce_residual(M, N):
        return {}
    nparts = car.nparts(M, N)
    ops = _serving_operands(rank, M, N, calls, dev)
    res0 = [_pattern(0, M * N, salt=300 + k).view(M, N).to(torch.bfloat16) for k in range(calls)]
    residuals = [r.to(dev).clone() for r in res0]
    parts = [torch.zeros(nparts * M, dtype=torch.float32, device=dev) for _ in range(calls)]
    wants, want_parts = [], []
    for k in range(calls):
        tot = res0[k].float() + sum(_pattern(r, M * N, dtype=torch.float32, salt=100 + k).view(M, N)
                                    for r in range(world))
        wants.append(tot.to(torch.bfloat16))
        want_parts.append(tot.view(M, nparts, N // nparts).pow(2).sum(-1).t().contiguous())

    def run_all():
        return [car.reduce_residual(ops[k], residuals[k], parts[k]) for k in range(calls)]

    def verify(outs) -> bool:
        ok = True
        for k in range(calls):
            ok &= _close(residuals[k], wants[k]) and tuple(outs[k].shape) == (nparts, M)
            ok &= bool(torch.equal(outs[k].float().cpu(), want_parts[k]))
        return ok

    def reset():
        for k in range(calls):
            residuals[k].copy_(res0[k].to(dev))
            parts[k].zero_()

    out: Dict[str, object] = {}
    outs = run_all()  # eager, back to back
    _sync(dev)
    out["eager"] = verify(outs)
    t0 = time.perf_counter()
    us = None
    if graph:
        reset()
        _sync(dev)
        side = torch.cuda.Stream(dev)
        side.wait_stream(torch.cuda.current_stream(dev))
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=side):
            gouts = run_all()
        _sync(dev)
        reset()  # (capture enqueues nothing; the replays below do the work)
        g.replay()
        _sync(dev)
        out["graph"] = verify(gouts)
        reset()
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        ev0.record()
        g.replay()
        ev1.record()
        _sync(dev)
        us = ev0.elapsed_time(ev1) * 1000.0 / calls
        out["graph_timed"] = verify(gouts)
        del g
    else:
        reset()
        t0 = time.perf_counter()
        outs = run_all()
        _sync(dev)
        us = (time.perf_counter() - t0) * 1e6 / calls
        out["repeat"] = verify(outs)
    return {"checks": out, "collective_us": round(us, 2) if us is not None else None,
            "shape": [M, N], "calls": calls}


def check_chunk_form(car, rank: int, world: int, dev: torch.device, M: int, N: int, chunks: int) -> Dict[str, bool]:
    """The column-chunk form of the fused collective (``reduce_residual_chunk``, the overlapped TP
    decode chain with POLYKEY_TP_DECODE_CHUNKS > 1): every chunk's own 2-slab operand,
    back to back, against the exact whole-width result."""
    if not (hasattr(car, "chunks_ok") and car.chunks_ok(M, N, chunks)):
        return {}
    Nc = N // chunks
    full = _pattern(rank, M * N, dtype=torch.float32, salt=400).view(M, N)
    res0 = _pattern(0, M * N, salt=401).view(M, N).to(torch.bfloat16)
    residual = res0.to(dev).clone()
    nparts = car.nparts(M, N)
    parts = torch.zeros(nparts * M, dtype=torch.float32, device=dev)
    for c in range(chunks):
        sl = full[:, c * Nc:(c + 1) * Nc]
        buf = torch.cat([(sl + 0.5).reshape(-1), torch.full((M * Nc,), -0.5)]).to(dev)
        car.reduce_residual_chunk(_Slabs(buf, 2, M, Nc), residual, parts, c, chunks)
    _sync(dev)
    tot = res0.float() + sum(_pattern(r, M * N, dtype=torch.float32, salt=400).view(M, N) for r in range(world))
    want_parts = tot.view(M, nparts, N // nparts).pow(2).sum(-1).t()
    return {f"chunks_{chunks}": _close(residual, tot.to(torch.bfloat16))
            and bool(torch.equal(parts.view(nparts, M).cpu(), want_parts))}


def check_push_form(car, rank: int, world: int, dev: torch.device, M: int, N: int) -> Dict[str, bool]:
    """The GEMM-epilogue push form (POLYKEY_TP_PUSH): a real MODE_PUSH decode GEMM at
    [M, K=512] x [N, K]^T whose weight selects column n % K of the rank-seeded activations (an exact
    product), its tiles pushed into the owners' slots, then ``reduce_residual_pushed``."""
    from ..ops import gemm
    if dev.type != "cuda" or not (hasattr(car, "push_ok") and car.push_ok(M, N, 64)):
        return {}
    K = 512
    x = _pattern(rank, M * K, salt=500).view(M, K).to(torch.bfloat16).to(dev)
    w = torch.zeros(N, K, dtype=torch.bfloat16)
    w[torch.arange(N), torch.arange(N) % K] = 1.0
    w = w.to(dev)
    wp = gemm.pack_weight(w)
    S, _ = gemm.partial_tiling(N, K, M, wp, True)
    ws = torch.empty(S * M * N, dtype=torch.float32, device=dev)
    counters = torch.zeros(N // 64, dtype=torch.int32, device=dev)
    res0 = _pattern(0, M * N, salt=501).view(M, N).to(torch.bfloat16)
    residual = res0.to(dev).clone()
    parts = torch.zeros((N // 256) * M, dtype=torch.float32, device=dev)
    nbc = gemm.push_projection(x, w, ws, wp, counters, car.push_target())
    p = car.reduce_residual_pushed(residual, parts, nbc)
    _sync(dev)
    cols = torch.arange(N) % K
    tot = res0.float() + sum(_pattern(r, M * K, salt=500).view(M, K).float()[:, cols] for r in range(world))
    want_parts = tot.view(M, N // 256, 256).pow(2).sum(-1).t()
    return {"push": _close(residual, tot.to(torch.bfloat16)) and bool(torch.equal(p.float().cpu(), want_parts))
            and int(counters.abs().sum()) == 0}


def check_ep_ipc(a2a, rank: int, world: int, dev: torch.device) -> Dict[str, bool]:
    """Dispatch + return of the IPC expert all-to-all: rank r sends (r + j) % 2 + 1 rows to rank j
    (expert id j + 10 * row), the owners return each row doubled."""
    H = a2a.H
    sends = [(rank + j) % 2 + 1 for j in range(world)]
    if sum(sends) > a2a.C:
        return {}
    rows = torch.cat([_pattern(rank, sends[j] * H, device=dev, salt=20 + j).view(-1, H) for j in range(world)])
    ids = torch.cat([torch.arange(sends[j], dtype=torch.int32) * 10 + j for j in range(world)]).to(dev)
    offs = torch.tensor([0] + list(torch.tensor(sends).cumsum(0)), dtype=torch.int32, device=dev)
    a2a.dispatch(rows.contiguous(), ids, offs)
    _sync(dev)
    ok = True
    for j in range(world):  # region j of this rank holds rank j's rows for this rank
        n = (j + rank) % 2 + 1
        got = a2a.recv_x[j * a2a.C: j * a2a.C + n]
        ok &= _close(got, _pattern(j, n * H, salt=20 + rank).view(-1, H))
        ok &= bool(torch.equal(a2a.recv_e[j * a2a.C: j * a2a.C + n].cpu(),
                               torch.arange(n, dtype=torch.int32) * 10 + rank))
    y = (a2a.recv_x.float() * 2).to(torch.bfloat16).contiguous()
    back = a2a.return_(y)
    _sync(dev)
    ok2 = _close(back[: rows.shape[0]], (rows.float() * 2).to(torch.bfloat16))
    return {"dispatch": bool(ok), "return": bool(ok2)}


# ------------------------------------------------------------------------------------- run
def _serving_check(st: ParallelState, serving: Tuple[int, int], report: dict, emit, verdict) -> None:
    """:func:`check_custom_ar_serving` under the watchdog, the fence-free protocol first.  When it
    fails on some rank and no rank saw a hang (the slot epochs are still in step), the whole group
    switches to the fenced protocol (custom_ar.set_fenced) and runs the check again; a second
    failure -- or a hang -- disables the custom collectives on every rank (RCCL takes over)."""
    from . import custom_ar as _car_mod
    car = st.custom_ar
    M, N = serving
    dev = st.device

    def off_car():
        car.close()
        st.custom_ar = None

    def attempt(name):
        holder = {}

        def fn():
            r = check_custom_ar_serving(car, st.tp_rank, st.tp_size, dev, M, N)
            holder.update(r)
            return dict(r.get("checks", {}))
        res, err = _guarded(name, fn, lambda: car.fail(), report, emit)
        if holder.get("collective_us") is not None:
            report.setdefault("collective_us", {})[name] = holder["collective_us"]
        report.setdefault("serving_shape", [M, N])
        return res, err

    name = "custom_ar_serving_fenced" if car.fenced else "custom_ar_serving"
    res, err = attempt(name)
    ok = bool(res) and all(res.values()) and err is None
    agreed = _agree(ok, st.tp_cpu_group, st.tp_size)
    if agreed or car.fenced or _car_mod.FENCED == "0":
        report["car_protocol"] = "fenced" if car.fenced else "fence-free"
        verdict(name, res, err, st.tp_cpu_group, st.tp_size, off_car)
        if st.custom_ar is not None:
            _optional_forms(st, car, M, N, report, emit, verdict)
        return
    # the fence-free form failed somewhere: record it, then retry fenced if every rank is still in step
    report["checks"][name] = {"ok": ok, "group_ok": False, **({"error": err} if err else {}), **res}
    clean = err is None and not (hasattr(car, "error") and car.error())
    if not _agree(clean, st.tp_cpu_group, st.tp_size):
        off_car()
        report["disabled"].append(name)
        return
    car.set_fenced(True)
    report["car_protocol"] = "fenced"
    res, err = attempt("custom_ar_serving_fenced")
    verdict("custom_ar_serving_fenced", res, err, st.tp_cpu_group, st.tp_size, off_car)
    if st.custom_ar is not None:
        _optional_forms(st, car, M, N, report, emit, verdict)


def _optional_forms(st: ParallelState, car, M: int, N: int, report: dict, emit, verdict) -> None:
    """The opt-in forms of the TP decode collective, checked when switched on: the
    column-chunk form (gemm.TP_DECODE_CHUNKS > 1) and the GEMM-epilogue push (gemm.TP_PUSH).  A
    failure turns that form off on every rank; the plain fused collective stays."""
    from ..ops import gemm
    dev = st.device
    M = min(M, 64)  # the push form takes one 64-row tile; the chunk form is row-agnostic
    forms = []
    if gemm.TP_DECODE_CHUNKS > 1:
        forms.append(("tp_decode_chunks", lambda: check_chunk_form(car, st.tp_rank, st.tp_size, dev, M, N,
                                                                   gemm.TP_DECODE_CHUNKS),
                      lambda: setattr(gemm, "TP_DECODE_CHUNKS", 1)))
    if gemm.TP_PUSH:
        forms.append(("tp_push", lambda: check_push_form(car, st.tp_rank, st.tp_size, dev, M, N),
                      lambda: setattr(gemm, "TP_PUSH", False)))
    for name, fn, off in forms:
        res, err = _guarded(name, fn, lambda: car.fail(), report, emit)
        verdict(name, res, err, st.tp_cpu_group, st.tp_size, off)



def _agree(ok: bool, group, world: int) -> bool:
    votes = [None] * world
    dist.all_gather_object(votes, bool(ok), group=group)
    return all(votes)


def _safe(fn: Callable[[], Dict[str, bool]]) -> Tuple[Dict[str, bool], Optional[str]]:
    try:
        return fn(), None
    except Exception as e:  # noqa: BLE001 - a raising path fails its check
        return {}, f"{type(e).__name__}: {e}"


# A check that has not returned after HANG_S seconds is hung (a collective whose peer never
# arrives, a device sync on a kernel that never ends).  The watchdog then records it, emits the
# report line at once (the log names the hung path even if nothing after it ever runs) and
# aborts the path (ncclCommAbort / the custom all-reduce's sticky error word), which makes the
# collective return; the check is failed and the group vote disables the path on every rank.
# A check still stuck GRACE_S after the abort ends the process: the line is printed again with
# "exit" and the process exits with HANG_EXIT -- never a silent hang, never an exec.
HANG_S = float(os.environ.get("POLYKEY_PREFLIGHT_HANG_S", "30"))
GRACE_S = float(os.environ.get("POLYKEY_PREFLIGHT_GRACE_S", "15"))
HANG_EXIT = 75


def _guarded(name: str, fn: Callable[[], Dict[str, bool]], abort: Callable[[], None], report: dict,
             emit: Callable[[str], None], hang_s: Optional[float] = None,
             grace_s: Optional[float] = None) -> Tuple[Dict[str, bool], Optional[str]]:
    """:func:`_safe` of ``fn`` under the hang watchdog (see HANG_S)."""
    hang_s = HANG_S if hang_s is None else hang_s
    grace_s = GRACE_S if grace_s is None else grace_s
    done = threading.Event()
    hung = threading.Event()

    def watch():
        if done.wait(hang_s):
            return
        hung.set()
        report.setdefault("hung", []).append(name)
        emit(json.dumps(report))
        try:
            abort()
        except Exception as e:  # noqa: BLE001 - the exit below is the backstop
            report.setdefault("abort_errors", {})[name] = f"{type(e).__name__}: {e}"
        if done.wait(grace_s):
            return
        report["exit"] = f"check {name!r} still hung {grace_s:.0f} s after its abort"
        emit(json.dumps(report))
        os._exit(HANG_EXIT)

    t = threading.Thread(target=watch, name=f"pk-preflight-watch-{name}", daemon=True)
    t.start()
    try:
        res, err = _safe(fn)
    finally:
        done.set()
    t.join()
    if hung.is_set():
        return res, f"hung: no result within {hang_s:.0f} s (path aborted)" + (f"; {err}" if err else "")
    return res, err


def peer_access(st: ParallelState) -> Optional[List[List[int]]]:
    """Row r: can rank r's device read each rank's device (hipDeviceCanAccessPeer)?  None when
    the ranks do not all see each other's devices (per-rank visibility) or run on the CPU."""
    if st.device.type != "cuda" or st.world_cpu_group is None:
        return None
    devs = [None] * st.world_size
    dist.all_gather_object(devs, st.device.index, group=st.world_cpu_group)
    n = torch.cuda.device_count()
    if any(d is None or d >= n for d in devs):
        row = None
    else:
        me = st.device.index
        row = [1 if d == me else int(torch.cuda.can_device_access_peer(me, d)) for d in devs]
    rows = [None] * st.world_size
    dist.all_gather_object(rows, row, group=st.world_cpu_group)
    return None if any(r is None for r in rows) else rows


def run(st: ParallelState, paths: Tuple[str, ...] = ("rccl", "custom_ar"), emit: Callable[[str], None] = None,
        serving: Optional[Tuple[int, int]] = None) -> dict:
    """Check every created device-collective path in ``paths`` ("rccl", "custom_ar", "ep_ipc",
    "custom_ar_serving" with ``serving`` = (rows, hidden)), disable the failed ones on every
    rank, return (and emit) the report."""
    t0 = time.perf_counter()
    report = {"event": "multi_gpu_preflight", "rank": st.rank, "world": st.world_size, "backend": st.backend,
              "ranks_per_device": st.ranks_per_device, "checks": {}, "disabled": []}
    emit = emit or (lambda s: print(s, file=sys.stderr, flush=True))
    if "rccl" in paths or "custom_ar" in paths:
        report["peer_access"] = peer_access(st)
    dev = st.device

    def _abort(obj, method):
        return lambda: getattr(obj, method)() if obj is not None and hasattr(obj, method) else None

    def verdict(name, res, err, group, world, disable):
        ok = bool(res) and all(res.values()) and err is None
        agreed = _agree(ok, group, world)
        report["checks"][name] = {"ok": ok, "group_ok": agreed, **({"error": err} if err else {}),
                                  **{k: v for k, v in res.items()}}
        if not agreed:
            disable()
            report["disabled"].append(name)

    if "rccl" in paths and st.rccl_tp is not None and st.tp_size > 1:
        rc = st.rccl_tp
        res, err = _guarded("rccl_tp", lambda: check_rccl(rc, st.tp_rank, st.tp_size, dev), _abort(rc, "abort"),
                            report, emit)

        def off_tp():
            if st.rccl_ep is st.rccl_tp:
                st.rccl_ep = None
            st.rccl_tp = None
        verdict("rccl_tp", res, err, st.tp_cpu_group, st.tp_size, off_tp)
    if "rccl" in paths and st.rccl_ep is not None and st.rccl_ep is not st.rccl_tp and st.ep_size > 1:
        rce = st.rccl_ep
        res, err = _guarded("rccl_ep", lambda: check_rccl(rce, st.ep_rank, st.ep_size, dev), _abort(rce, "abort"),
                            report, emit)
        verdict("rccl_ep", res, err, st.ep_cpu_group, st.ep_size, lambda: setattr(st, "rccl_ep", None))
    if "custom_ar" in paths and st.custom_ar is not None:
        car = st.custom_ar
        res, err = _guarded("custom_ar", lambda: check_custom_ar(car, st.tp_rank, st.tp_size, dev),
                            _abort(car, "fail"), report, emit)

        def off_car():
            car.close()
            st.custom_ar = None
        verdict("custom_ar", res, err, st.tp_cpu_group, st.tp_size, off_car)
    if "custom_ar_serving" in paths and st.custom_ar is not None and serving is not None:
        _serving_check(st, serving, report, emit, verdict)
    if "ep_ipc" in paths and st.ep_a2a is not None:
        a2a = st.ep_a2a
        res, err = _guarded("ep_ipc", lambda: check_ep_ipc(a2a, st.ep_rank, st.ep_size, dev), _abort(a2a, "fail"),
                            report, emit)

        def off_ep():
            for x in (st.ep_a2a, st.ep_a2a_prefill):
                if x is not None:
                    x.close()
            st.ep_a2a = st.ep_a2a_prefill = None
        verdict("ep_ipc", res, err, st.ep_cpu_group, st.ep_size, off_ep)
    report["seconds"] = round(time.perf_counter() - t0, 3)
    if st.rank == 0 or report["disabled"] or any(not c["ok"] for c in report["checks"].values()):
        emit(json.dumps(report))
    return report
