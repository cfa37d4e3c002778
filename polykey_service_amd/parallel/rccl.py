"""Direct RCCL communicators through the native binding ``csrc/comm/rccl_comm.hip``.

SURVEY.md §2.3 / §5.8: RCCL "through a C++ wrapper that enqueues on our own HIP streams,
unique-id bootstrap over torch.distributed".  ``torch.distributed``'s "nccl" backend is RCCL too,
but every call goes through ProcessGroupNCCL: an internal collective stream, an event wait from
the caller's stream and one back, a work object per call.  :class:`RcclComm` issues the RCCL call
on the caller's current stream -- the compute stream, the comm stream of an overlapped prefill
projection, or a stream under HIP-graph capture -- and nothing else.

Used for the expert-parallel all-to-all (dispatch / combine, ``parallel/comm.py``) and for TP
all-reduces too large for the one-shot xGMI kernel when ``init_parallel`` runs on RCCL
(``POLYKEY_RCCL_DIRECT=0`` keeps everything on torch.distributed).  The library resolves the
RCCL copy PyTorch already loaded, so the process holds one RCCL.

Failure handling: :meth:`RcclComm.check` polls the communicator's asynchronous
error without blocking and raises; :meth:`RcclComm.abort` tears a hung communicator down.
"""
from __future__ import annotations

import ctypes
import math
import threading
from typing import List, Optional, Sequence

import torch
import torch.distributed as dist

from .._native.loader import load_cdll

_P, _I, _SZ = ctypes.c_void_p, ctypes.c_int, ctypes.c_size_t
_lock = threading.Lock()
_state = {"lib": None, "loaded": None}

DTYPES = {torch.bfloat16: 0, torch.float32: 1, torch.int32: 2, torch.uint8: 3, torch.float16: 4, torch.int64: 5}
OPS = {"sum": 0, "max": 1, "min": 2}


class RcclError(RuntimeError):
    pass


def _lib() -> ctypes.CDLL:
    with _lock:
        if _state["lib"] is None:
            lib = load_cdll("libpk_comm")
            lib.pk_rccl_load.argtypes = [ctypes.c_char_p]
            lib.pk_rccl_library.restype = ctypes.c_char_p
            lib.pk_rccl_error_string.argtypes = [_I]
            lib.pk_rccl_error_string.restype = ctypes.c_char_p
            lib.pk_rccl_unique_id.argtypes = [_P]
            lib.pk_rccl_init.argtypes = [ctypes.POINTER(_P), _P, _I, _I]
            for n in ("pk_rccl_destroy", "pk_rccl_abort", "pk_rccl_async_error"):
                getattr(lib, n).argtypes = [_P]
            lib.pk_rccl_all_reduce.argtypes = [_P, _P, _P, _SZ, _I, _I, _P]
            lib.pk_rccl_all_gather.argtypes = [_P, _P, _P, _SZ, _I, _P]
            lib.pk_rccl_reduce_scatter.argtypes = [_P, _P, _P, _SZ, _I, _I, _P]
            lib.pk_rccl_broadcast.argtypes = [_P, _P, _P, _SZ, _I, _I, _P]
            arr = ctypes.POINTER(_SZ)
            lib.pk_rccl_all_to_allv.argtypes = [_P, _P, arr, arr, _P, arr, arr, _I, _I, _P]
            _state["lib"] = lib
        return _state["lib"]


def load(path: Optional[str] = None) -> bool:
    """Resolve RCCL (the copy already in the process first); True when usable."""
    lib = _lib()
    if _state["loaded"] is None or (not _state["loaded"] and path):
        _state["loaded"] = lib.pk_rccl_load(path.encode() if path else None) == 0
    return bool(_state["loaded"])


def library() -> str:
    return _lib().pk_rccl_library().decode() if load() else ""


def version() -> int:
    """RCCL version code (e.g. 22703 = 2.27.3), -1 when RCCL cannot be loaded."""
    return _lib().pk_rccl_version() if load() else -1


def _check(rc: int, what: str) -> None:
    if rc != 0:
        msg = _lib().pk_rccl_error_string(rc)
        raise RcclError(f"{what} failed ({rc}: {msg.decode() if msg else '?'})")


def unique_id() -> bytes:
    if not load():
        raise RcclError("RCCL library not available")
    buf = ctypes.create_string_buffer(_lib().pk_rccl_unique_id_size())
    _check(_lib().pk_rccl_unique_id(buf), "ncclGetUniqueId")
    return bytes(buf.raw)


def _sizes(vals: Sequence[int]):
    return (_SZ * len(vals))(*[int(v) for v in vals])


class RcclComm:
    """One RCCL communicator of ``nranks`` ranks; this process is ``rank`` on ``device``."""

    def __init__(self, uid: bytes, nranks: int, rank: int, device: torch.device):
        if not load():
            raise RcclError("RCCL library not available")
        self.nranks, self.rank, self.device = nranks, rank, device
        self.lib = _lib()
        h = _P()
        with torch.cuda.device(device):
            _check(self.lib.pk_rccl_init(ctypes.byref(h), ctypes.create_string_buffer(uid, len(uid)), nranks, rank),
                   "ncclCommInitRank")
        self.comm = h

    @classmethod
    def create(cls, group=None, device: Optional[torch.device] = None, cpu_group=None) -> "RcclComm":
        """Collective over ``group``: its first rank draws the unique id, the id travels over
        ``cpu_group`` (default: ``group``) as a pickled object, every rank joins."""
        device = device or torch.device("cuda", torch.cuda.current_device())
        n = dist.get_world_size(group)
        r = dist.get_rank(group)
        obj = [unique_id() if r == 0 else None]
        src = dist.get_global_rank(group, 0) if group is not None else 0
        dist.broadcast_object_list(obj, src=src, group=cpu_group if cpu_group is not None else group)
        return cls(obj[0], n, r, device)

    @classmethod
    def single(cls, device: Optional[torch.device] = None) -> "RcclComm":
        """A one-rank communicator (no rendezvous): exercises the binding on one GPU."""
        device = device or torch.device("cuda", torch.cuda.current_device())
        return cls(unique_id(), 1, 0, device)

    # ------------------------------------------------------------------ helpers
    def _stream(self) -> int:
        return torch.cuda.current_stream(self.device).cuda_stream

    @staticmethod
    def _dt(t: torch.Tensor) -> int:
        if t.dtype not in DTYPES:
            raise TypeError(f"RCCL binding: unsupported dtype {t.dtype}")
        return DTYPES[t.dtype]

    def _ok(self) -> None:
        if self.comm is None:
            raise RcclError("communicator closed")

    # -------------------------------------------------------------- collectives
    def all_reduce(self, x: torch.Tensor, op: str = "sum", out: Optional[torch.Tensor] = None) -> torch.Tensor:
        """Element-wise reduction over the ranks (``out`` may be ``x``: in place)."""
        self._ok()
        if not x.is_contiguous():
            raise ValueError("all_reduce needs a contiguous tensor")
        out = torch.empty_like(x) if out is None else out
        if not out.is_contiguous() or out.numel() != x.numel():
            raise ValueError("all_reduce: out must be contiguous and match x")
        _check(self.lib.pk_rccl_all_reduce(self.comm, x.data_ptr(), out.data_ptr(), x.numel(), self._dt(x), OPS[op],
                                           self._stream()), "ncclAllReduce")
        return out

    def all_gather(self, x: torch.Tensor, out: Optional[torch.Tensor] = None) -> torch.Tensor:
        """[n, ...] per rank -> [nranks * n, ...] in rank order (``out``: contiguous destination)."""
        self._ok()
        x = x.contiguous()
        if out is None:
            out = torch.empty((self.nranks * x.shape[0],) + tuple(x.shape[1:]), dtype=x.dtype, device=x.device)
        elif not out.is_contiguous() or out.numel() != self.nranks * x.numel():
            raise ValueError("all_gather: out must be contiguous with nranks x the input's elements")
        _check(self.lib.pk_rccl_all_gather(self.comm, x.data_ptr(), out.data_ptr(), x.numel(), self._dt(x),
                                           self._stream()), "ncclAllGather")
        return out

    def reduce_scatter(self, x: torch.Tensor, op: str = "sum", out: Optional[torch.Tensor] = None) -> torch.Tensor:
        """[nranks * n, ...] per rank -> this rank's [n, ...] block of the reduction."""
        self._ok()
        x = x.contiguous()
        if x.shape[0] % self.nranks:
            raise ValueError("reduce_scatter: dim 0 must divide by the rank count")
        if out is None:
            out = torch.empty((x.shape[0] // self.nranks,) + tuple(x.shape[1:]), dtype=x.dtype, device=x.device)
        elif not out.is_contiguous() or out.numel() * self.nranks != x.numel():
            raise ValueError("reduce_scatter: out must be contiguous with 1/nranks of the input's elements")
        _check(self.lib.pk_rccl_reduce_scatter(self.comm, x.data_ptr(), out.data_ptr(), out.numel(), self._dt(x),
                                               OPS[op], self._stream()), "ncclReduceScatter")
        return out

    def broadcast(self, x: torch.Tensor, root: int = 0) -> torch.Tensor:
        """In place: every rank's ``x`` becomes rank ``root``'s."""
        self._ok()
        if not x.is_contiguous():
            raise ValueError("broadcast needs a contiguous tensor (it works in place)")
        _check(self.lib.pk_rccl_broadcast(self.comm, x.data_ptr(), x.data_ptr(), x.numel(), self._dt(x), root,
                                          self._stream()), "ncclBroadcast")
        return x

    def all_to_allv(self, x: torch.Tensor, out_splits: List[int], in_splits: List[int]) -> torch.Tensor:
        """Rows of ``x`` (dim 0) split by ``in_splits`` go to ranks 0..n-1; rank j's rows for
        this rank arrive in ``out_splits[j]`` rows, concatenated in rank order."""
        self._ok()
        if len(out_splits) != self.nranks or len(in_splits) != self.nranks:
            raise ValueError("all_to_allv: one split per rank")
        if sum(in_splits) != x.shape[0]:
            raise ValueError("all_to_allv: in_splits must cover dim 0 of x")
        x = x.contiguous()
        row = math.prod(x.shape[1:])  # 0-row inputs (an idle EP rank) are valid
        out = torch.empty((sum(out_splits),) + tuple(x.shape[1:]), dtype=x.dtype, device=x.device)
        sc = [s * row for s in in_splits]
        rc = [s * row for s in out_splits]
        sd = [sum(sc[:j]) for j in range(self.nranks)]
        rd = [sum(rc[:j]) for j in range(self.nranks)]
        _check(self.lib.pk_rccl_all_to_allv(self.comm, x.data_ptr(), _sizes(sc), _sizes(sd), out.data_ptr(),
                                            _sizes(rc), _sizes(rd), self.nranks, self._dt(x), self._stream()),
               "all_to_allv (grouped ncclSend/ncclRecv)")
        return out

    # ------------------------------------------------------------ health / life
    def check(self) -> None:
        """Raise if RCCL recorded an asynchronous error on this communicator (non-blocking)."""
        if self.comm is not None:
            _check(self.lib.pk_rccl_async_error(self.comm), "RCCL communicator")

    def abort(self) -> None:
        """Tear the communicator down even while one of its collectives is hung."""
        if self.comm is not None:
            self.lib.pk_rccl_abort(self.comm)
            self.comm = None

    def close(self) -> None:
        if self.comm is not None:
            with torch.cuda.device(self.device):
                self.lib.pk_rccl_destroy(self.comm)
            self.comm = None
