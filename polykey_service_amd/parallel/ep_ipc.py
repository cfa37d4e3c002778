"""Expert all-to-all over xGMI peer memory (csrc/comm/ep_alltoall.hip) for DP attention + EP.

Decode-sized MoE layers exchange token rows through fixed-capacity per-peer regions of IPC
buffers: a dispatch kernel writes each rank's destination-sorted rows straight into the owners'
receive regions and a return kernel writes the expert outputs back into the senders' buffers in
the order they were sent.  Counts and offsets stay on the device -- no ``.cpu()`` per layer, no
RCCL host split lists -- so a DP-attention + EP decode step is one HIP graph (VERDICT r2 item 4,
SURVEY.md §5.8).  Prefill-sized steps (more rows than the capacity) keep the RCCL all-to-all.

Capacity ``C`` = rows one rank may send to one peer in a call = max decode batch x top-k; the
receive side holds W x C rows of H bf16 (Mixtral, 8 ranks, batch 256: 8 x 512 x 4096 x 2 B =
32 MiB per rank).
"""
from __future__ import annotations

import ctypes
import logging
import os
from typing import Optional

import torch
import torch.distributed as dist

from .._native.loader import load_cdll

log = logging.getLogger(__name__)
_P, _I, _LL = ctypes.c_void_p, ctypes.c_int, ctypes.c_longlong


def _lib() -> ctypes.CDLL:
    lib = load_cdll("libpk_comm")
    if not getattr(lib, "_pk_ep_typed", False):
        lib.pk_ep_create.argtypes = [_I, _I, _LL, _LL]
        lib.pk_ep_create.restype = _P
        lib.pk_ep_get_handle.argtypes = [_P, _P]
        lib.pk_ep_open.argtypes = [_P, _P]
        for n in ("pk_ep_recv_x", "pk_ep_recv_e", "pk_ep_ret_x"):
            getattr(lib, n).argtypes = [_P]
            getattr(lib, n).restype = _P
        lib.pk_ep_dispatch.argtypes = [_P, _P, _P, _P, _P]
        lib.pk_ep_return.argtypes = [_P, _P, _P]
        lib.pk_ep_check_error.argtypes = [_P]
        lib.pk_ep_set_error.argtypes = [_P]
        lib.pk_ep_set_timeout_ms.argtypes = [_P, _LL]
        lib.pk_ep_destroy.argtypes = [_P]
        lib.pk_ep_destroy.restype = None
        lib._pk_ep_typed = True
    return lib


class EpAllToAllError(RuntimeError):
    """An EP peer did not arrive at an expert all-to-all within the timeout."""


class EpAllToAll:
    def __init__(self, cpu_group, rank: int, world: int, device: torch.device, capacity: int, hidden: int,
                 timeout_s: Optional[float] = None):
        self.lib = _lib()
        self.rank, self.world, self.device = rank, world, device
        self.C, self.H = capacity, hidden
        self.ctx = None
        hsz = self.lib.pk_ep_ipc_handle_size()
        # a rank whose local setup failed still joins the handle exchange (with None): no peer
        # blocks in it, and every rank raises together
        mine, err = None, None
        try:
            with torch.cuda.device(device):
                self.ctx = self.lib.pk_ep_create(rank, world, capacity, hidden)
            if not self.ctx:
                raise RuntimeError("pk_ep_create failed")
            t = timeout_s if timeout_s is not None else float(os.environ.get("POLYKEY_CUSTOM_AR_TIMEOUT_S", "30"))
            self.lib.pk_ep_set_timeout_ms(self.ctx, max(1, int(t * 1000)))
            buf = ctypes.create_string_buffer(hsz)
            if self.lib.pk_ep_get_handle(self.ctx, buf) != 0:
                raise RuntimeError("hipIpcGetMemHandle failed")
            mine = bytes(buf.raw)
        except Exception as e:  # noqa: BLE001 - re-raised after the exchange
            err = e
        allh = [None] * world
        dist.all_gather_object(allh, mine, group=cpu_group)
        if err is not None or any(h is None for h in allh):
            self.close()
            raise err if err is not None else RuntimeError("an EP peer could not create its IPC regions")
        blob = ctypes.create_string_buffer(b"".join(allh), hsz * world)
        with torch.cuda.device(device):
            rc = self.lib.pk_ep_open(self.ctx, blob)
        if rc != 0:
            raise RuntimeError(f"pk_ep_open failed ({rc})")
        # this rank's regions as tensors (fixed addresses: graph-safe)
        self.recv_x = _wrap(self.lib.pk_ep_recv_x(self.ctx), (world * capacity, hidden), torch.bfloat16, device)
        self.recv_e = _wrap(self.lib.pk_ep_recv_e(self.ctx), (world * capacity,), torch.int32, device)
        self.ret_x = _wrap(self.lib.pk_ep_ret_x(self.ctx), (capacity, hidden), torch.bfloat16, device)

    def fits(self, rows: int) -> bool:
        """A call whose every rank sends at most ``rows`` rows in total fits the regions."""
        return rows <= self.C

    def dispatch(self, send_x: torch.Tensor, send_e: torch.Tensor, offsets: torch.Tensor) -> None:
        """send_x [n, H] bf16 destination-sorted, send_e [n] int32 expert ids local to their
        destination, offsets [W + 1] int32 (device).  After it, ``recv_x`` / ``recv_e`` hold every
        peer's rows (region src = rows [src * C, src * C + n_src); padding ids are -1)."""
        assert send_x.is_contiguous() and send_x.dtype == torch.bfloat16 and send_x.shape[-1] == self.H
        assert send_e.dtype == torch.int32 and offsets.dtype == torch.int32 and offsets.numel() == self.world + 1
        assert send_x.shape[0] <= self.C, "more rows than the expert all-to-all capacity"
        rc = self.lib.pk_ep_dispatch(self.ctx, send_x.data_ptr(), send_e.data_ptr(), offsets.data_ptr(),
                                     torch.cuda.current_stream(self.device).cuda_stream)
        if rc != 0:
            raise RuntimeError(f"expert dispatch launch failed ({rc})")

    def return_(self, y: torch.Tensor) -> torch.Tensor:
        """y [W * C, H] bf16: outputs for the received rows in arrival order.  Returns this rank's
        [C, H] view of its own rows back, in the order it sent them."""
        assert y.is_contiguous() and y.shape == (self.world * self.C, self.H) and y.dtype == torch.bfloat16
        rc = self.lib.pk_ep_return(self.ctx, y.data_ptr(), torch.cuda.current_stream(self.device).cuda_stream)
        if rc != 0:
            raise RuntimeError(f"expert return launch failed ({rc})")
        return self.ret_x

    def error(self) -> int:
        return self.lib.pk_ep_check_error(self.ctx)

    def check(self) -> None:
        if self.ctx and self.lib.pk_ep_check_error(self.ctx):
            raise EpAllToAllError(f"expert all-to-all: an EP peer of rank {self.rank} did not arrive within the "
                                  "timeout (group failed; restart the job)")

    def fail(self) -> None:
        if self.ctx:
            self.lib.pk_ep_set_error(self.ctx)

    def close(self) -> None:
        if self.ctx:
            self.lib.pk_ep_destroy(self.ctx)
            self.ctx = None


def _wrap(ptr: int, shape, dtype, device) -> torch.Tensor:
    """A tensor view of device memory owned by the native context (kept alive by it)."""
    n = 1
    for s in shape:
        n *= s
    nbytes = n * torch.empty((), dtype=dtype).element_size()

    class _Holder:
        __cuda_array_interface__ = {"shape": (nbytes,), "typestr": "|u1", "data": (ptr, False), "version": 3}
    raw = torch.as_tensor(_Holder(), device=device)
    return raw.view(dtype).view(*shape)


def maybe_create(st, capacity: int, hidden: int) -> Optional[EpAllToAll]:
    """IPC expert all-to-all for a DP-attention + EP group whose ranks share one node."""
    if os.environ.get("POLYKEY_EP_IPC", "1") == "0" or not st.dp_attention or st.device.type != "cuda":
        return None
    if st.ep_size > 8 or int(os.environ.get("LOCAL_WORLD_SIZE", str(st.world_size))) < st.ep_size:
        return None
    a2a, err = None, None
    try:
        a2a = EpAllToAll(st.ep_cpu_group, st.ep_rank, st.ep_size, st.device, capacity, hidden)
    except Exception as e:  # noqa: BLE001 - RCCL all-to-all stays
        err = e
    # all ranks on the IPC path or none: a subset on IPC would spin on flags the others never set
    votes = [None] * st.ep_size
    dist.all_gather_object(votes, a2a is not None, group=st.ep_cpu_group)
    if all(votes):
        return a2a
    log.warning("IPC expert all-to-all unavailable (%s); using RCCL", err or "failed on a peer")
    if a2a is not None:
        a2a.close()
    return None
