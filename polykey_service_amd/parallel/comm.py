"""Tensor-parallel / expert-parallel collectives.

Device collectives go through ``torch.distributed`` on the TP group, which is RCCL over
xGMI on MI355X (backend "nccl"); the same code runs on gloo in CPU tests.  Per-call sizes
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
    dist.all_reduce(x, group=st.tp_group)
    return x


_COMM_STREAMS = {}


def _comm_stream(device: torch.device) -> "torch.cuda.Stream":
    s = _COMM_STREAMS.get(device)
    if s is None:
        s = _COMM_STREAMS[device] = torch.cuda.Stream(device)
    return s


OVERLAP_MIN_ROWS = int(os.environ.get("POLYKEY_TP_OVERLAP_MIN_ROWS", "256"))


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


def tp_all_gather_last(x: torch.Tensor) -> torch.Tensor:
    """[.., n] per rank → [.., n * tp] (rank-major along the last dim)."""
    st = get_state()
    if st.tp_size == 1:
        return x
    x = x.contiguous()
    out = torch.empty((st.tp_size * x.shape[0],) + tuple(x.shape[1:]), dtype=x.dtype, device=x.device)
    dist.all_gather_into_tensor(out, x, group=st.tp_group)
    out = out.view((st.tp_size,) + tuple(x.shape))
    return out.movedim(0, -2).reshape(*x.shape[:-1], x.shape[-1] * st.tp_size)


def tp_all_to_all(x: torch.Tensor, out_splits: List[int], in_splits: List[int]) -> torch.Tensor:
    """Variable-size all-to-all along dim 0 (MoE expert dispatch/combine)."""
    st = get_state()
    if st.tp_size == 1:
        return x
    out = torch.empty((sum(out_splits),) + tuple(x.shape[1:]), dtype=x.dtype, device=x.device)
    dist.all_to_all_single(out, x.contiguous(), out_splits, in_splits, group=st.tp_group)
    return out


def tp_all_to_all_counts(counts: torch.Tensor) -> torch.Tensor:
    """Exchange per-destination token counts (int64 [tp]) → counts received from each rank."""
    st = get_state()
    if st.tp_size == 1:
        return counts
    out = torch.empty_like(counts)
    dist.all_to_all_single(out, counts.contiguous(), group=st.tp_group)
    return out


def tp_broadcast_object(obj=None):
    """Control plane: TP leader → other ranks of its group (gloo, CPU)."""
    st = get_state()
    if st.tp_size == 1:
        return obj
    lst = [obj]
    src = st.dp_rank * st.tp_size
    dist.broadcast_object_list(lst, src=src, group=st.tp_cpu_group)
    return lst[0]


def tp_broadcast_tensor(t: torch.Tensor) -> torch.Tensor:
    st = get_state()
    if st.tp_size == 1:
        return t
    dist.broadcast(t, src=st.dp_rank * st.tp_size, group=st.tp_cpu_group if not t.is_cuda else st.tp_group)
    return t


def barrier(group: Optional[object] = None) -> None:
    if dist.is_initialized():
        dist.barrier(group=group)
