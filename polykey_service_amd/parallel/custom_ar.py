"""One-shot / two-shot all-reduce over xGMI peer memory (csrc/comm/custom_allreduce.hip).

For the small activations of TP decode (a 70B TP=8 step issues 160 all-reduces of ~1 MiB,
SURVEY.md §6) a single kernel in which every rank reads every peer's buffer over xGMI beats
RCCL's ring/tree latency.  The group's IPC buffers are exchanged once over the gloo control
group; messages larger than the buffer, non-bf16 tensors, or a failed start-up self-test fall
back to RCCL (``dist.all_reduce``).  ``POLYKEY_CUSTOM_AR=0`` disables it; ``force`` also
enables it on a gloo-backed GPU group (tests run TP ranks that share one GPU that way).

Failure detection: every wait in the kernel is bounded by a wall-clock timeout
(``POLYKEY_CUSTOM_AR_TIMEOUT_S``, default 30 s).  A peer that misses it sets a sticky error word
in host-mapped memory; :meth:`CustomAllReduce.error` reads it without a GPU sync and the model
runner checks it after every step, raising :class:`CustomAllReduceError` — the engine loop dies,
health goes NOT_SERVING and the server exits non-zero for its supervisor to restart.
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
# grid of the fused decode collective (0: one workgroup per (row, owner-chunk group), <= 512); A/B knob
_FUSED_BLOCKS = int(os.environ.get("POLYKEY_CAR_FUSED_BLOCKS", "0"))
# slot protocol: "auto" = fence-free until the serving-shape preflight finds a mismatch on this
# group's devices (then fenced, parallel/preflight.py); "1" = fenced from the start; "0" = never fenced
FENCED = os.environ.get("POLYKEY_CAR_FENCED", "auto")
# the largest buffer the kernels' 32-bit buffer offsets address (csrc pk_car_create)
MAX_DATA_BYTES = (0x7FFFFFF0 - (1 << 20)) // 4


def _lib() -> ctypes.CDLL:
    lib = load_cdll("libpk_comm")
    if not getattr(lib, "_pk_typed", False):
        lib.pk_car_create.argtypes = [_I, _I, _LL]
        lib.pk_car_create.restype = _P
        lib.pk_car_get_handle.argtypes = [_P, _P]
        lib.pk_car_open.argtypes = [_P, _P]
        lib.pk_car_allreduce_bf16.argtypes = [_P, _P, _P, _LL, _I, _P]
        lib.pk_car_allreduce_bf16_algo.argtypes = [_P, _P, _P, _LL, _I, _I, _P]
        lib.pk_car_allgather.argtypes = [_P, _P, _P, _LL, _LL, _I, _P]
        lib.pk_car_reduce_residual.argtypes = [_P, _P, _I, _P, _P, _P, _I, _I, _I, _P]
        lib.pk_car_reduce_residual_nparts.argtypes = [_P, _I, _I]
        lib.pk_car_reduce_residual_ex.argtypes = [_P, _P, _I, _P, _P, _P, _I, _I, _I, _I, _I, _P]
        lib.pk_car_push_target.argtypes = [_P, ctypes.POINTER(_P), ctypes.POINTER(_I), ctypes.POINTER(_I),
                                           ctypes.POINTER(_LL)]
        lib.pk_car_reduce_residual_pushed.argtypes = [_P, _P, _P, _I, _I, _I, _I, _P]
        lib.pk_car_sig_bytes.restype = _LL
        lib.pk_car_create_loopback.argtypes = [_I, _I, _LL]
        lib.pk_car_create_loopback.restype = _P
        lib.pk_car_check_error.argtypes = [_P]
        lib.pk_car_clear_error.argtypes = [_P]
        lib.pk_car_set_error.argtypes = [_P]
        lib.pk_car_set_timeout_ms.argtypes = [_P, _LL]
        lib.pk_car_set_fenced.argtypes = [_P, _I]
        lib.pk_car_device_ctx.argtypes = [_P, _P, _I]
        lib.pk_car_get_fenced.argtypes = [_P]
        lib.pk_car_destroy.argtypes = [_P]
        lib.pk_car_destroy.restype = None
        lib._pk_typed = True
    return lib


class CustomAllReduceError(RuntimeError):
    """A TP peer did not arrive at a custom all-reduce within the timeout."""


class CustomAllReduce:
    def __init__(self, cpu_group, rank: int, world: int, device: torch.device, max_bytes: int = 16 << 20,
                 blocks: int = 0, timeout_s: Optional[float] = None):
        self.lib = _lib()
        self.rank, self.world, self.device = rank, world, device
        if not 0 < max_bytes <= MAX_DATA_BYTES:
            raise ValueError(f"custom all-reduce slot of {max_bytes} bytes: 32-bit slot offsets allow "
                             f"at most {MAX_DATA_BYTES}")
        self.max_bytes = max_bytes
        self.blocks = blocks
        # grid of the fused decode collective (0: one workgroup per (row, 1024-column chunk), up
        # to 512).  Ranks sharing ONE GPU (rehearsals, tests) need every rank's grid resident at
        # once: maybe_create caps it there.
        self.fused_blocks = _FUSED_BLOCKS
        self.ctx = None
        hsz = self.lib.pk_car_ipc_handle_size()
        # the local half (allocation, IPC handle) never skips the handle exchange: a rank that
        # failed still reaches the all-gather (with None), so no peer blocks in it, and every rank
        # then raises together
        mine, err = None, None
        try:
            with torch.cuda.device(device):
                self.ctx = self.lib.pk_car_create(rank, world, max_bytes)
            if not self.ctx:
                raise RuntimeError("pk_car_create failed (uncached IPC buffer allocation)")
            if timeout_s is None:
                timeout_s = float(os.environ.get("POLYKEY_CUSTOM_AR_TIMEOUT_S", "30"))
            self.set_timeout(timeout_s)
            self.set_fenced(FENCED == "1")
            buf = ctypes.create_string_buffer(hsz)
            if self.lib.pk_car_get_handle(self.ctx, buf) != 0:
                raise RuntimeError("hipIpcGetMemHandle failed")
            mine = bytes(buf.raw)
        except Exception as e:  # noqa: BLE001 - re-raised after the exchange
            err = e
        allh = [None] * world
        dist.all_gather_object(allh, mine, group=cpu_group)
        if err is not None or any(h is None for h in allh):
            self.close()
            raise err if err is not None else RuntimeError("a TP peer could not create its IPC buffers")
        blob = ctypes.create_string_buffer(b"".join(allh), hsz * world)
        with torch.cuda.device(device):
            rc = self.lib.pk_car_open(self.ctx, blob)
        if rc != 0:
            raise RuntimeError(f"pk_car_open failed ({rc})")

    @classmethod
    def loopback(cls, rank: int, world: int, device: torch.device, max_bytes: int = 16 << 20) -> "CustomAllReduce":
        """One-process stand-in group for timing the real collective kernels (tools/tp_solo.py
        --car loopback; csrc pk_car_create_loopback): peers are local buffers whose flags never
        block.  The reduced values are meaningless; the kernels' own work is all there."""
        self = cls.__new__(cls)
        self.lib = _lib()
        self.rank, self.world, self.device = rank, world, device
        self.max_bytes, self.blocks, self.fused_blocks = max_bytes, 0, _FUSED_BLOCKS
        with torch.cuda.device(device):
            self.ctx = self.lib.pk_car_create_loopback(rank, world, max_bytes)
        if not self.ctx:
            raise RuntimeError("pk_car_create_loopback failed")
        self.set_fenced(FENCED == "1")
        return self

    @property
    def fenced(self) -> bool:
        """The fenced slot protocol is in use (release / acquire fences around every flag)."""
        return bool(self.ctx) and self.lib.pk_car_get_fenced(self.ctx) == 1

    def set_fenced(self, on: bool) -> None:
        """Switch this rank's context to the fenced (``on``) or fence-free slot protocol for
        every later call.  Every rank of the group must switch together (preflight does)."""
        if self.lib.pk_car_set_fenced(self.ctx, 1 if on else 0) != 0:
            raise RuntimeError("pk_car_set_fenced failed")

    def supports(self, x: torch.Tensor) -> bool:
        n = x.numel() * x.element_size()
        return (x.is_cuda and x.dtype == torch.bfloat16 and x.is_contiguous() and n % 16 == 0
                and 0 < n <= self.max_bytes)

    def all_reduce(self, x: torch.Tensor, out: Optional[torch.Tensor] = None, algo: int = 0) -> torch.Tensor:
        """algo: 0 = by size (one-shot <= 512 KiB, two-shot above), 1 = one-shot, 2 = two-shot."""
        out = torch.empty_like(x) if out is None else out
        rc = self.lib.pk_car_allreduce_bf16_algo(self.ctx, x.data_ptr(), out.data_ptr(),
                                                 x.numel() * x.element_size(), self.blocks, algo,
                                                 torch.cuda.current_stream(self.device).cuda_stream)
        if rc != 0:
            raise RuntimeError(f"custom all-reduce launch failed ({rc})")
        return out

    def supports_gather(self, x: torch.Tensor) -> bool:
        """[rows, cols] with 16-byte rows that fit one slot (LM-head logits of a decode step)."""
        if not (x.is_cuda and x.dim() == 2 and x.is_contiguous()):
            return False
        row = x.shape[1] * x.element_size()
        return row % 16 == 0 and 0 < x.shape[0] * row <= self.max_bytes

    def all_gather_last(self, x: torch.Tensor) -> torch.Tensor:
        """[rows, cols] per rank -> [rows, world * cols], rank-major along the last dim."""
        out = torch.empty((x.shape[0], self.world * x.shape[1]), dtype=x.dtype, device=x.device)
        rc = self.lib.pk_car_allgather(self.ctx, x.data_ptr(), out.data_ptr(), x.shape[0],
                                       x.shape[1] * x.element_size(), self.blocks,
                                       torch.cuda.current_stream(self.device).cuda_stream)
        if rc != 0:
            raise RuntimeError(f"custom all-gather launch failed ({rc})")
        return out

    def supports_reduce_residual(self, M: int, N: int) -> bool:
        """Shapes the fused decode collective takes (:meth:`reduce_residual`)."""
        return M > 0 and N % 1024 == 0 and M * N * 2 <= self.max_bytes

    def nparts(self, M: int, N: int) -> int:
        """Rows of the norm parts :meth:`reduce_residual` writes for an [M, N] residual: N / 256
        (two-shot form) or N / 1024 (one-shot)."""
        return int(self.lib.pk_car_reduce_residual_nparts(self.ctx, M, N))

    def reduce_residual(self, pending, residual: torch.Tensor, parts: torch.Tensor) -> torch.Tensor:
        """Fused TP collective of a row-parallel decode projection, one launch: this rank's
        split-K slabs (a :class:`~polykey_service_amd.ops.gemm.Partial`) or bf16 partial [M, N]
        are reduced locally, summed over the group through the IPC slots (rank order), added
        into ``residual`` in place, and ``parts`` receives per-column-chunk sums of squares of
        the new residual ([nparts, M] view returned) for the next folded-norm projection.  With
        4+ ranks the collective is two-shot (reduce-scatter to the owner of each 256-column
        chunk, then all-gather: ~2 (W-1)/W of the message over xGMI per rank instead of
        (W-1)x; parts per 256 columns), else one-shot (parts per 1024 columns)."""
        M, N = residual.shape
        if not (residual.is_contiguous() and residual.dtype == torch.bfloat16 and self.supports_reduce_residual(M, N)):
            raise ValueError(f"reduce_residual: unsupported residual {tuple(residual.shape)} {residual.dtype}")
        nparts = self.lib.pk_car_reduce_residual_nparts(self.ctx, M, N)
        assert parts.numel() >= nparts * M and parts.dtype == torch.float32
        if isinstance(pending, torch.Tensor):
            assert pending.shape == (M, N) and pending.is_contiguous() and pending.dtype == torch.bfloat16
            slabs, S, partial = 0, 0, pending.data_ptr()
        else:
            assert pending.M == M and pending.N == N and pending.buf.numel() >= pending.S * M * N
            slabs, S, partial = pending.buf.data_ptr(), pending.S, 0
        rc = self.lib.pk_car_reduce_residual(self.ctx, slabs, S, partial, residual.data_ptr(), parts.data_ptr(), M, N,
                                             self.fused_blocks, torch.cuda.current_stream(self.device).cuda_stream)
        if rc != 0:
            raise RuntimeError(f"fused TP reduce launch failed ({rc})")
        return parts.view(-1)[: nparts * M].view(nparts, M)

    def chunks_ok(self, M: int, N: int, chunks: int) -> bool:
        """Can the fused collective of an [M, N] residual run as ``chunks`` column chunks with the
        same norm-parts layout as the whole (both forms: chunk widths multiples of 1024)?"""
        if chunks < 2 or N % (1024 * chunks) or not self.supports_reduce_residual(M, N):
            return False
        return self.nparts(M, N // chunks) * chunks == self.nparts(M, N)

    def reduce_residual_chunk(self, pending, residual: torch.Tensor, parts: torch.Tensor, chunk: int,
                              chunks: int) -> None:
        """:meth:`reduce_residual` of column chunk ``chunk`` of ``chunks``: ``pending`` (a
        ``gemm.Partial``) holds that chunk's own slabs [S, M, N / chunks]; the chunk's columns of
        ``residual`` and its rows of the norm parts are updated.  Same arithmetic per element as
        the whole-width call (bit-identical).  The TP decode chain runs one per chunk on the comm
        stream while the compute stream runs the next chunk's GEMM (models/llama.py)."""
        M, N = residual.shape
        if not (residual.is_contiguous() and residual.dtype == torch.bfloat16 and self.chunks_ok(M, N, chunks)):
            raise ValueError(f"reduce_residual_chunk: unsupported residual {tuple(residual.shape)} / {chunks}")
        Nc = N // chunks
        assert pending.M == M and pending.N == Nc and pending.S >= 1 and 0 <= chunk < chunks
        npc = self.nparts(M, Nc)
        assert parts.numel() >= npc * chunks * M and parts.dtype == torch.float32
        rc = self.lib.pk_car_reduce_residual_ex(
            self.ctx, pending.buf.data_ptr(), pending.S, None, residual.data_ptr() + chunk * Nc * 2,
            parts.data_ptr() + chunk * npc * M * 4, M, Nc, N, Nc, self.fused_blocks,
            torch.cuda.current_stream(self.device).cuda_stream)
        if rc != 0:
            raise RuntimeError(f"fused TP reduce (chunk {chunk}) launch failed ({rc})")

    def device_ctx(self):
        """This rank's collective context as the kernels see it (csrc/comm/car_device.h CarDev, a
        byte buffer): what a launch of the kernel library that carries the two-shot collective
        takes (gemm.linear_partial_rowscale_car).  Re-read after :meth:`set_fenced`."""
        n = int(self.lib.pk_car_device_ctx_size())
        buf = ctypes.create_string_buffer(n)
        if self.lib.pk_car_device_ctx(self.ctx, buf, n) != 0:
            raise RuntimeError("pk_car_device_ctx failed")
        return buf

    def carry_ok(self, M: int, N: int) -> bool:
        """Shapes a consumer launch can carry this collective for (the two-shot form at W = 4 / 8,
        one 64-row tile): kernels/car_gemm.hip."""
        return (self.world in (4, 8) and 0 < M <= 64 and N % (256 * self.world) == 0
                and self.nparts(M, N) == N // 256 and M * (N // (256 * self.world)) <= 1024)

    def push_target(self):
        """Where a decode GEMM's push epilogue writes (gemm.push_projection)."""
        if getattr(self, "_push_target", None) is None:
            from ..ops.gemm import PushTarget
            peers, rank, world, nbytes = _P(), _I(), _I(), _LL()
            if self.lib.pk_car_push_target(self.ctx, ctypes.byref(peers), ctypes.byref(rank), ctypes.byref(world),
                                           ctypes.byref(nbytes)) != 0:
                raise RuntimeError("pk_car_push_target failed")
            self._push_target = PushTarget(peers.value, rank.value, world.value, nbytes.value)
        return self._push_target

    def push_ok(self, M: int, N: int, nbc: int = 128) -> bool:
        """Shapes the pushed collective takes: the two-shot layout (parts per 256 columns, what
        :meth:`nparts` gives the consumers), one 64-row tile, n-blocks the flag rows index."""
        return (not self.fenced and 0 < M <= 64 and N % (256 * self.world) == 0 and N // nbc <= 1024
                and M * N * 2 + (N // 256) * M * 4 <= self.max_bytes and self.nparts(M, N) == N // 256)

    def reduce_residual_pushed(self, residual: torch.Tensor, parts: torch.Tensor, nbc: int) -> torch.Tensor:
        """:meth:`reduce_residual` after a push GEMM (gemm.push_projection): every rank's bf16
        partial of this rank's chunks is already in this rank's slot, so the collective starts at
        the reduce-scatter.  Same residual and parts bits as the two-shot :meth:`reduce_residual`."""
        M, N = residual.shape
        if not (residual.is_contiguous() and residual.dtype == torch.bfloat16 and self.push_ok(M, N, nbc)):
            raise ValueError(f"reduce_residual_pushed: unsupported residual {tuple(residual.shape)} {residual.dtype}")
        nparts = N // 256
        assert parts.numel() >= nparts * M and parts.dtype == torch.float32
        rc = self.lib.pk_car_reduce_residual_pushed(self.ctx, residual.data_ptr(), parts.data_ptr(), M, N, nbc,
                                                    self.fused_blocks,
                                                    torch.cuda.current_stream(self.device).cuda_stream)
        if rc != 0:
            raise RuntimeError(f"pushed TP reduce launch failed ({rc})")
        return parts.view(-1)[: nparts * M].view(nparts, M)

    def set_timeout(self, seconds: float) -> None:
        self.lib.pk_car_set_timeout_ms(self.ctx, max(1, int(seconds * 1000)))

    def error(self) -> int:
        """1 once a wait timed out (sticky; host-mapped word, no GPU sync)."""
        return self.lib.pk_car_check_error(self.ctx)

    def check(self) -> None:
        """Raise :class:`CustomAllReduceError` if a peer has timed out (called every engine step)."""
        if self.ctx and self.lib.pk_car_check_error(self.ctx):
            raise CustomAllReduceError(f"custom all-reduce: a TP peer of rank {self.rank} did not arrive within "
                                       "the timeout (group failed; restart the job)")

    def fail(self) -> None:
        """Mark this rank's group failed (the failure path's abort): every later call returns at
        once without waiting and :meth:`check` raises."""
        if self.ctx:
            self.lib.pk_car_set_error(self.ctx)

    def clear_error(self) -> None:
        """Tests only: re-arm after a deliberately provoked timeout."""
        self.lib.pk_car_clear_error(self.ctx)

    def self_test(self) -> bool:
        """Rank-dependent pattern reduced twice (both buffer parities) and checked on the host."""
        ok = True
        for it in range(2):
            n = 4096 * (it + 1) + 8
            x = torch.full((n,), float(self.rank + 1 + it), dtype=torch.bfloat16, device=self.device)
            y = self.all_reduce(x)
            torch.cuda.synchronize(self.device)
            want = sum(r + 1 + it for r in range(self.world))
            ok &= bool((y.float() == want).all().item())
        return ok and self.error() == 0

    def close(self) -> None:
        if self.ctx:
            self.lib.pk_car_destroy(self.ctx)
            self.ctx = None


def maybe_create(st) -> Optional[CustomAllReduce]:
    """Custom all-reduce for this rank's TP group when it is a single-node GPU group."""
    if os.environ.get("POLYKEY_CUSTOM_AR", "1") == "0" or st.tp_size < 2 or st.device.type != "cuda":
        return None
    if st.tp_size > 8 or int(os.environ.get("LOCAL_WORLD_SIZE", str(st.world_size))) < st.tp_size:
        return None
    # every rank reaches the same collectives whatever fails where: the constructor's handle
    # exchange, an open vote, the self-test vote (all ranks keep the IPC path or none does)
    car, err = None, None
    try:
        car = CustomAllReduce(st.tp_cpu_group, st.tp_rank, st.tp_size, st.device)
    except Exception as e:  # noqa: BLE001 - any failure → RCCL path
        err = e
    if not _all_ranks(car is not None, st.tp_cpu_group, st.tp_size):
        log.warning("custom all-reduce unavailable (%s); using RCCL", err or "failed on a peer")
        if car is not None:
            car.close()
        return None
    if st.shared_device:
        car.fused_blocks = 64  # ranks share a GPU: every rank's grid must be resident at once
    good = False
    try:
        good = car.self_test()
    except Exception as e:  # noqa: BLE001
        log.warning("custom all-reduce self-test raised (%s)", e)
    if _all_ranks(good, st.tp_cpu_group, st.tp_size):
        return car
    log.warning("custom all-reduce self-test failed on some rank; using RCCL")
    car.close()
    return None


def _all_ranks(ok: bool, cpu_group, world: int) -> bool:
    """All-or-none vote over the group's gloo control group."""
    votes = [None] * world
    dist.all_gather_object(votes, bool(ok), group=cpu_group)
    return all(votes)
