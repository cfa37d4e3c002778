"""Prefill-sized GEMMs on the hand-written MFMA kernel (``csrc/kernels/gemm_prefill.hip``).

``y = x @ W^T`` (``W`` in PyTorch ``[N, K]`` layout), bf16 in / fp32 accumulate / bf16 out, for
hundreds to tens of thousands of rows; dense, or grouped by expert with the group row offsets
read on the device (MoE prefill: no host read-back, one launch per projection, graph
capturable).  Optional fused SiLU(gate) * up for gate/up rows interleaved in blocks of 16
(:func:`polykey_service_amd.ops.gemm.interleave_gate_up`).

CPU tensors use the fp32 reference with the kernel's bf16 rounding points.
"""
from __future__ import annotations

import ctypes
import os
from typing import Optional

import torch

from . import native

BM = 256
BN = 256
# 6: the 4-wave, one-wave-per-SIMD kernel (AGPR accumulators, BK 64, buffer_load ... lds staging
# into a 3-slot A / 2-slot W ring; K % 128 == 0), 4: the 8-wave ping-pong kernel (the fallback for
# K % 128 != 0) -- csrc/kernels/gemm_prefill.hip.  Round 6: 7-16 % faster than the round-5 kernel;
# hipBLASLt 6-9 % ahead on the dense shapes, 21 % behind on the grouped w2
# (profiles/r6_prefill_gemm_buffer_lds.md, r4_prefill_gemm_4wave.md)
VARIANT = 6


class PrefillGemmArgs(ctypes.Structure):
    """Mirror of ``struct PrefillGemmArgs`` (checked against ``pk_prefill_gemm_args_size``)."""
    _fields_ = [("C", ctypes.c_void_p), ("A", ctypes.c_void_p), ("W", ctypes.c_void_p),
                ("M", ctypes.c_int), ("N", ctypes.c_int), ("K", ctypes.c_int), ("lda", ctypes.c_int),
                ("ldc", ctypes.c_int), ("row_offsets", ctypes.c_void_p), ("w_stride", ctypes.c_longlong),
                ("groups", ctypes.c_int), ("tiles_m", ctypes.c_int), ("silu", ctypes.c_int)]


_checked = False


def supported(N: int, K: int) -> bool:
    return N % BN == 0 and K % 64 == 0


def _launch(a: PrefillGemmArgs, variant: Optional[int] = None) -> None:
    global _checked
    lib = native.lib()
    if not _checked:
        fn = lib.pk_prefill_gemm_args_size
        fn.restype = ctypes.c_int
        n = fn()
        assert n == ctypes.sizeof(PrefillGemmArgs), f"PrefillGemmArgs mismatch: C {n} vs ctypes {ctypes.sizeof(PrefillGemmArgs)}"
        f = lib.pk_prefill_gemm
        f.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p]
        f.restype = ctypes.c_int
        _checked = True
    v = VARIANT if variant is None else variant
    if v >= 6 and a.K % 128:
        v = 4 + v % 2  # the 8-wave kernel needs only K % 64 == 0
    native.check(lib.pk_prefill_gemm(ctypes.byref(a), v, native.stream_ptr()), "pk_prefill_gemm")


def _ref(x: torch.Tensor, w: torch.Tensor, silu: bool) -> torch.Tensor:
    y = (x.float() @ w.float().t()).to(torch.bfloat16).float()
    if silu:
        v = y.view(y.shape[0], -1, 2, 16)
        g, u = v[:, :, 0].reshape(y.shape[0], -1), v[:, :, 1].reshape(y.shape[0], -1)
        y = torch.nn.functional.silu(g).to(torch.bfloat16).float() * u
    return y.to(x.dtype)


def linear(x: torch.Tensor, w: torch.Tensor, out: Optional[torch.Tensor] = None, silu: bool = False,
           variant: Optional[int] = None, packed: Optional[torch.Tensor] = None) -> torch.Tensor:
    """x [M, K] @ w[N, K]^T -> [M, N] (SiLU: [M, N/2]), optionally into ``out``.  ``packed``:
    :func:`~polykey_service_amd.ops.gemm.pack_weight` of ``w`` is read instead (``w`` then only
    gives the shape: a model holding only the packed copy passes a placeholder)."""
    M, K = x.shape
    N = w.shape[0]
    n_out = N // 2 if silu else N
    if not x.is_cuda:
        if packed is not None:
            from .gemm import unpack_weight
            w = unpack_weight(packed)
        y = _ref(x, w, silu)
        if out is None:
            return y
        out.copy_(y)
        return out
    if out is None:
        out = torch.empty((M, n_out), dtype=x.dtype, device=x.device)
    if M == 0:
        return out
    src = packed if packed is not None else w
    if (not supported(N, K) or x.stride(1) != 1 or not src.is_contiguous() or out.stride(1) != 1
            or (packed is not None and (K % 128 or tuple(packed.shape) != (N, K)))):
        raise ValueError(f"prefill GEMM: unsupported shape/layout M={M} N={N} K={K}")
    if packed is not None and variant not in (5, 7):
        variant = VARIANT + 1  # the same kernels reading the decode GEMM's block-packed W
    a = PrefillGemmArgs()
    a.C, a.A, a.W = out.data_ptr(), x.data_ptr(), src.data_ptr()
    a.M, a.N, a.K, a.lda, a.ldc = M, N, K, x.stride(0), out.stride(0)
    a.groups, a.tiles_m, a.silu = 0, (M + BM - 1) // BM, int(silu)
    _launch(a, variant)
    return out


def grouped_linear(x: torch.Tensor, w: torch.Tensor, offsets: torch.Tensor, silu: bool = False,
                   out: Optional[torch.Tensor] = None, variant: Optional[int] = None) -> torch.Tensor:
    """Rows [offsets[e], offsets[e+1]) of ``x`` times ``w[e]^T`` (w: [G, N, K], offsets int32 on
    the device, rows past offsets[G] untouched).  One launch; the grid covers
    ceil(rows / 256) + G tile rows and the kernel maps each to its group."""
    T, K = x.shape
    G, N, _ = w.shape
    n_out = N // 2 if silu else N
    if not x.is_cuda:
        offs = offsets.tolist()
        y = torch.zeros((T, n_out), dtype=x.dtype) if out is None else out
        for e in range(G):
            lo, hi = offs[e], offs[e + 1]
            if hi > lo:
                y[lo:hi] = _ref(x[lo:hi], w[e], silu)
        return y
    if out is None:
        out = torch.empty((T, n_out), dtype=x.dtype, device=x.device)
    if T == 0:
        return out
    if not supported(N, K) or x.stride(1) != 1 or not w.is_contiguous() or offsets.dtype != torch.int32:
        raise ValueError(f"grouped prefill GEMM: unsupported shape/layout T={T} N={N} K={K}")
    a = PrefillGemmArgs()
    a.C, a.A, a.W = out.data_ptr(), x.data_ptr(), w.data_ptr()
    a.M, a.N, a.K, a.lda, a.ldc = T, N, K, x.stride(0), out.stride(0)
    a.row_offsets, a.w_stride, a.groups = offsets.data_ptr(), N * K, G
    a.tiles_m, a.silu = (T + BM - 1) // BM + G, int(silu)
    _launch(a, variant)
    return out
