"""Tensor-parallel / expert-parallel collectives.

Device collectives are RCCL over xGMI on MI355X: the direct communicators of
``parallel/rccl.py`` (one RCCL call on the caller's stream) when ``init_parallel`` created them,
else ``torch.distributed`` on the TP / EP group (backend "nccl"); the same code runs on gloo in
CPU tests.  Small decode all-reduces / gathers take the one-shot xGMI kernel instead.  Per-call sizes
for the north-star configs (SURVEY.md §2.3 collective table): 70B TP8 decode all-reduces
[B, 8192] bf16 = 16 KiB·B twice per layer — latency-bound, hence HIP-graph capture of the
whole decode step (RCCL collectives are graph-capturable); prefill all-reduces are tens of
MiB and bandwidth-bound over the 7 xGMI links.
"""
from __future__ import annotations

import os
from typing import List, Optional

import torch
import torch.distributed as dist

from .state import get_state


def tp_all_reduce(x: torch.Tensor) -> torch.Tensor:
    """Sum over the TP group, in place (returns ``x``)."""
    st = get_state()
    if st.tp_size == 1:
        return x
    car = st.custom_ar
    if car is not None and car.supports(x):
        return car.all_reduce(x, out=x)  # one-shot xGMI kernel (small decode messages)
    rc = _direct(st.rccl_tp, x)
    if rc is not None and x.is_contiguous():
        return rc.all_reduce(x, out=x)
    dist.all_reduce(x, group=st.tp_group)
    return x


def _direct(comm, x: torch.Tensor):
    """The direct RCCL communicator for a device tensor, or None (torch.distributed / gloo)."""
    return comm if comm is not None and x.is_cuda else None


_COMM_STREAMS = {}


def _comm_stream(device: torch.device) -> "torch.cuda.Stream":
    s = _COMM_STREAMS.get(device)
    if s is None:
        s = _COMM_STREAMS[device] = torch.cuda.Stream(device)
    return s


def comm_stream(device: torch.device) -> "torch.cuda.Stream":
    """The dedicated HIP stream collectives overlap compute on (one per device)."""
    return _comm_stream(device)


OVERLAP_MIN_ROWS = 256
# row chunks of an overlapped prefill projection: with 2 at best half of each collective hides
# under the next chunk's GEMM; 4 where every chunk keeps >= OVERLAP_MIN_ROWS rows
OVERLAP_MAX_CHUNKS = int(os.environ.get("POLYKEY_OVERLAP_CHUNKS", "4"))


def overlap_chunks(T: int) -> int:
    """Row chunks for a T-token overlapped prefill collective (1: no overlap)."""
    c = 1
    while c * 2 <= OVERLAP_MAX_CHUNKS and T >= c * 2 * OVERLAP_MIN_ROWS:
        c *= 2
    return c


def tp_row_parallel_overlapped(x: torch.Tensor, n_out: int, fn, chunks: int = 2,
                               min_rows: Optional[int] = None) -> torch.Tensor:
    """``all_reduce(fn(x))`` for a row-parallel projection with the collective of chunk i on a
    dedicated HIP stream while the GEMM of chunk i+1 runs on the compute stream (prefill-sized
    ``x``; SURVEY.md §2.3 TP: RCCL all-reduce overlapped with the GEMMs).  ``fn(rows, out)``
    writes the local partial product of ``rows`` into ``out``."""
    st = get_state()
    T = x.shape[0]
    out = torch.empty((T, n_out), dtype=x.dtype, device=x.device)
    min_rows = OVERLAP_MIN_ROWS if min_rows is None else min_rows
    if st.tp_size == 1 or not x.is_cuda or T < min_rows * chunks:
        fn(x, out)
        return tp_all_reduce(out)
    main = torch.cuda.current_stream(x.device)
    cs = _comm_stream(x.device)
    bounds = [T * i // chunks for i in range(chunks + 1)]
    for i in range(chunks):
        sl = slice(bounds[i], bounds[i + 1])
        fn(x[sl], out[sl])
        cs.wait_stream(main)
        with torch.cuda.stream(cs):
            tp_all_reduce(out[sl])
    main.wait_stream(cs)
    out.record_stream(cs)
    return out


# ---------------------------------------------------------------- sequence parallelism
# Megatron-style SP for TP prefill (SURVEY.md §2.3 "SP"): the residual stream is sharded by
# token between the row-parallel projections (reduce-scatter) and the column-parallel ones
# (all-gather), so RMSNorm and the residual adds run on 1/tp of the rows and each rank holds
# 1/tp of the residual.  Same bytes on xGMI as the all-reduce it replaces (RS + AG), but the
# two halves overlap with different GEMMs: the reduce-scatter of row chunk c runs on the comm
# stream while the row-parallel GEMM of chunk c+1 runs, and the all-gather of chunk c+1 runs
# while the column-parallel GEMM of chunk c does.
#
# Layout: ``Tp`` = T padded to a multiple of tp*chunks, chunk c = rows [c*Tc, (c+1)*Tc) with
# Tc = Tp/chunks; rank r's shard is [chunks, Tc/tp] rows, chunk c's piece being rows
# c*Tc + r*Tc/tp + [0, Tc/tp).  Row-wise ops (norm, residual add) do not care about the order.


class SPLayout:
    __slots__ = ("T", "Tp", "chunks", "tp", "rank")

    def __init__(self, T: int, chunks: int = 1):
        st = get_state()
        self.T, self.chunks, self.tp, self.rank = T, chunks, st.tp_size, st.tp_rank
        q = self.tp * chunks
        self.Tp = (T + q - 1) // q * q

    @property
    def rows(self) -> int:
        """Rows of one rank's shard."""
        return self.Tp // self.tp

    def chunk(self, c: int):
        Tc = self.Tp // self.chunks
        return c * Tc, (c + 1) * Tc, c * Tc // self.tp, (c + 1) * Tc // self.tp


def _reduce_scatter(out: torch.Tensor, x: torch.Tensor) -> None:
    st = get_state()
    rc = _direct(st.rccl_tp, x)
    if rc is not None and out.is_contiguous():
        rc.reduce_scatter(x, out=out)
        return
    if dist.get_backend(st.tp_group) != "gloo":
        dist.reduce_scatter_tensor(out, x, group=st.tp_group)
        return
    t = x.clone()  # gloo has no reduce-scatter: all-reduce and keep this rank's slice
    dist.all_reduce(t, group=st.tp_group)
    out.copy_(t.view((st.tp_size, -1) + tuple(x.shape[1:]))[st.tp_rank])


def sp_reduce_scatter(y: torch.Tensor, lay: SPLayout, fn=None) -> torch.Tensor:
    """Row-parallel partials → this rank's summed shard [lay.rows, n].  ``fn(rows, out)``:
    compute the partial of x-rows ``rows`` into ``out`` chunk by chunk (``y`` = the input x)
    so the collective of chunk c overlaps the GEMM of chunk c+1; ``fn=None``: ``y`` is the
    finished [T, n] partial."""
    T, tp = lay.T, lay.tp
    n = y.shape[1] if fn is None else fn.n_out
    full = torch.empty((lay.Tp, n), dtype=y.dtype, device=y.device)
    if lay.Tp > T:
        full[T:].zero_()
    shard = torch.empty((lay.rows, n), dtype=y.dtype, device=y.device)
    overlap = y.is_cuda and lay.chunks > 1
    main = torch.cuda.current_stream(y.device) if overlap else None
    cs = _comm_stream(y.device) if overlap else None
    for c in range(lay.chunks):
        lo, hi, slo, shi = lay.chunk(c)
        rhi = min(hi, T)
        if rhi > lo:
            if fn is None:
                full[lo:rhi].copy_(y[lo:rhi])
            else:
                fn(y[lo:rhi], full[lo:rhi])
        if overlap:
            cs.wait_stream(main)
            with torch.cuda.stream(cs):
                _reduce_scatter(shard[slo:shi], full[lo:hi])
        else:
            _reduce_scatter(shard[slo:shi], full[lo:hi])
    if overlap:
        main.wait_stream(cs)
        full.record_stream(cs)
    return shard


def sp_all_gather(shard: torch.Tensor, lay: SPLayout, fn=None) -> torch.Tensor:
    """Shards → the full [T, n] rows on every rank.  ``fn(rows, out)``: a column-parallel
    projection applied chunk by chunk as soon as that chunk has arrived (the gather of chunk
    c+1 overlaps it); returns its [T, fn.n_out] output instead."""
    st = get_state()
    T = lay.T
    full = torch.empty((lay.Tp, shard.shape[1]), dtype=shard.dtype, device=shard.device)
    overlap = shard.is_cuda and lay.chunks > 1 and fn is not None
    main = torch.cuda.current_stream(shard.device) if overlap else None
    cs = _comm_stream(shard.device) if overlap else None
    events = []
    if overlap:
        cs.wait_stream(main)
    rc = _direct(st.rccl_tp, shard)

    def gather(dst, src):
        if rc is not None:
            rc.all_gather(src, out=dst)
        else:
            dist.all_gather_into_tensor(dst, src, group=st.tp_group)
    for c in range(lay.chunks):
        lo, hi, slo, shi = lay.chunk(c)
        if overlap:
            with torch.cuda.stream(cs):
                gather(full[lo:hi], shard[slo:shi])
                ev = torch.cuda.Event()
                ev.record(cs)
            events.append(ev)
        else:
            gather(full[lo:hi], shard[slo:shi])
    if overlap:
        full.record_stream(cs)
        shard.record_stream(cs)
    if fn is None:
        return full[:T]
    out = torch.empty((T, fn.n_out), dtype=shard.dtype, device=shard.device)
    for c in range(lay.chunks):
        lo, hi, _, _ = lay.chunk(c)
        hi = min(hi, T)
        if overlap:
            main.wait_event(events[c])
        if hi > lo:
            fn(full[lo:hi], out[lo:hi])
    return out


class RowsFn:
    """``fn(rows, out)`` with its output width, for :func:`sp_reduce_scatter` / :func:`sp_all_gather`."""
    __slots__ = ("f", "n_out")

    def __init__(self, f, n_out: int):
        self.f, self.n_out = f, n_out

    def __call__(self, rows, out):
        self.f(rows, out)


def tp_all_gather_last(x: torch.Tensor) -> torch.Tensor:
    """[.., n] per rank → [.., n * tp] (rank-major along the last dim).  Decode-sized 2-D
    inputs (the LM head's logits) go through the IPC all-gather kernel, so a TP decode step's
    graph holds no collective-library call (parallel/custom_ar.py)."""
    st = get_state()
    if st.tp_size == 1:
        return x
    x = x.contiguous()
    car = st.custom_ar
    if car is not None and car.supports_gather(x):
        return car.all_gather_last(x)
    out = torch.empty((st.tp_size * x.shape[0],) + tuple(x.shape[1:]), dtype=x.dtype, device=x.device)
    rc = _direct(st.rccl_tp, x)
    if rc is not None:
        rc.all_gather(x, out=out)
    else:
        dist.all_gather_into_tensor(out, x, group=st.tp_group)
    out = out.view((st.tp_size,) + tuple(x.shape))
    return out.movedim(0, -2).reshape(*x.shape[:-1], x.shape[-1] * st.tp_size)


def tp_all_to_all(x: torch.Tensor, out_splits: List[int], in_splits: List[int]) -> torch.Tensor:
    """Variable-size all-to-all along dim 0 (MoE expert dispatch/combine)."""
    st = get_state()
    if st.tp_size == 1:
        return x
    rc = _direct(st.rccl_tp, x)
    if rc is not None:
        return rc.all_to_allv(x, out_splits, in_splits)
    out = torch.empty((sum(out_splits),) + tuple(x.shape[1:]), dtype=x.dtype, device=x.device)
    dist.all_to_all_single(out, x.contiguous(), out_splits, in_splits, group=st.tp_group)
    return out


def tp_all_to_all_counts(counts: torch.Tensor) -> torch.Tensor:
    """Exchange per-destination token counts (int64 [tp]) → counts received from each rank."""
    st = get_state()
    if st.tp_size == 1:
        return counts
    rc = _direct(st.rccl_tp, counts)
    if rc is not None:
        return rc.all_to_allv(counts.reshape(-1, 1), [1] * st.tp_size, [1] * st.tp_size).view(-1)
    out = torch.empty_like(counts)
    dist.all_to_all_single(out, counts.contiguous(), group=st.tp_group)
    return out


def ep_all_to_all(x: torch.Tensor, out_splits: List[int], in_splits: List[int]) -> torch.Tensor:
    """Variable-size all-to-all along dim 0 over the expert-parallel group."""
    st = get_state()
    if st.ep_size == 1:
        return x
    if x.is_cuda and dist.get_backend(st.ep_group) == "gloo":
        # ranks sharing one GPU (rehearsal / tests): gloo moves host copies
        return ep_all_to_all(x.cpu(), out_splits, in_splits).to(x.device)
    rc = _direct(st.rccl_ep, x)
    if rc is not None:  # one group of ncclSend/ncclRecv pairs on the compute stream
        return rc.all_to_allv(x, out_splits, in_splits)
    out = torch.empty((sum(out_splits),) + tuple(x.shape[1:]), dtype=x.dtype, device=x.device)
    dist.all_to_all_single(out, x.contiguous(), out_splits, in_splits, group=st.ep_group)
    return out


def ep_all_to_all_counts(counts: torch.Tensor) -> torch.Tensor:
    """Per-destination row counts (int64 [ep]) → counts received from each EP rank."""
    st = get_state()
    if st.ep_size == 1:
        return counts
    if counts.is_cuda and dist.get_backend(st.ep_group) == "gloo":
        return ep_all_to_all_counts(counts.cpu()).to(counts.device)
    rc = _direct(st.rccl_ep, counts)
    if rc is not None:
        return rc.all_to_allv(counts.reshape(-1, 1), [1] * st.ep_size, [1] * st.ep_size).view(-1)
    out = torch.empty_like(counts)
    dist.all_to_all_single(out, counts.contiguous(), group=st.ep_group)
    return out


def ep_vote(busy: bool, stopping: bool = False, ntok: int = 0):
    """Lockstep vote of the DP-attention ranks → (any rank busy, every rank stopping, the largest
    token count).  One node: the shared-memory vote board (µs); else one gloo all-reduce."""
    st = get_state()
    if st.ep_size == 1 or st.ep_cpu_group is None:
        return bool(busy), bool(stopping), int(ntok)
    if st.ep_board is not None:
        from ..engine.model_runner import peer_timeout_ms
        return st.ep_board.vote(bool(busy), bool(stopping), int(ntok), max(peer_timeout_ms(), 600000))
    t = torch.tensor([1 if busy else 0, 0 if stopping else 1, int(ntok)], dtype=torch.int64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX, group=st.ep_cpu_group)
    return bool(t[0].item()), not bool(t[1].item()), int(t[2].item())


def ep_any(flag: bool) -> bool:
    """True if any DP-attention rank's flag is set (one lockstep vote)."""
    return ep_vote(flag)[0]


def tp_broadcast_object(obj=None):
    """Control plane: TP leader → other ranks of its group (gloo, CPU)."""
    st = get_state()
    if st.tp_size == 1:
        return obj
    lst = [obj]
    src = st.tp_leader
    dist.broadcast_object_list(lst, src=src, group=st.tp_cpu_group)
    return lst[0]


def tp_broadcast_tensor(t: torch.Tensor) -> torch.Tensor:
    st = get_state()
    if st.tp_size == 1:
        return t
    rc = _direct(st.rccl_tp, t)
    if rc is not None and t.is_contiguous():
        return rc.broadcast(t, root=0)  # the group's first rank is its leader
    dist.broadcast(t, src=st.tp_leader, group=st.tp_cpu_group if not t.is_cuda else st.tp_group)
    return t


def barrier(group: Optional[object] = None) -> None:
    if dist.is_initialized():
        dist.barrier(group=group)
