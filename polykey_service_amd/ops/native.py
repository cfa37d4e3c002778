"""ctypes binding of the gfx950 kernel library ``libpk_kernels.so`` (``csrc/kernels``).

Every launcher takes raw device pointers plus the caller's HIP stream
(``torch.cuda.current_stream().cuda_stream``), so launches are ordered with torch's own
work and are captured by HIP graphs.  A launcher returns 0 on success, a negative value for
an unsupported shape, or a HIP error code; :func:`check` turns non-zero into an exception.

Policy: on a GPU tensor the HIP kernel is the *only* path — if the library cannot be loaded
the op raises (:func:`lib`), it never silently falls back to a PyTorch composition.  CPU
tensors (unit tests in this GPU-less container) use the fp32 PyTorch reference in
:mod:`polykey_service_amd.ops.reference`.
"""
from __future__ import annotations

import ctypes
import threading
from typing import Optional

import torch

from .._native.loader import load_cdll

_lib: Optional[ctypes.CDLL] = None
_lock = threading.Lock()

P = ctypes.c_void_p
I32 = ctypes.c_int
I64 = ctypes.c_int64
F32 = ctypes.c_float

# name -> argtypes (restype is always c_int)
SIGNATURES = {
    "pk_kernels_abi_version": [],
    "pk_rmsnorm": [P, P, P, I32, I32, I32, I32, F32, P],
    "pk_fused_add_rmsnorm": [P, P, P, I32, I32, F32, P],
    "pk_silu_and_mul": [P, P, I32, I32, P],
    "pk_rope_and_cache": [P, P, P, P, P, P, I32, I32, I32, I32, I32, I32, I32, P],
    "pk_paged_decode": [P, P, P, P, P, P, P, P, I32, I32, I32, I32, I32, I32, I32, F32, I32, P],
    "pk_set_decode_z": [I32],
    "pk_set_decode_fill": [I32],
    "pk_paged_decode_qkv": [P, P, I32, I32, P, P, P, P, P, P, P, P, P, I32, I32, I32, I32, I32, I32, F32, I32, P],
    "pk_paged_prefill": [P, P, P, P, P, P, P, P, I32, I32, I32, I32, I32, I32, I32, I32, F32, P],
    "pk_sample": [P, P, P, P, P, P, P, P, P, I32, I32, I32, I32, P],
    "pk_embedding": [P, P, P, I32, I32, I32, I32, P],
    "pk_moe_topk_softmax": [P, P, P, I32, I32, I32, I32, I32, P],
    "pk_moe_align": [P, P, P, P, I32, I32, I32, I32, P],
    "pk_moe_permute": [P, P, P, P, I32, I32, I32, I32, P],
    "pk_moe_unpermute": [P, P, P, P, I32, I32, I32, P],
    "pk_moe_gemm": [P, P, P, P, I32, I32, I32, I32, I32, I32, P],
    "pk_moe_unpermute_partial": [P, P, I32, I32, P, P, I32, I32, I32, P],
    "pk_moe_combine_add_rmsnorm": [P, P, P, P, P, P, I32, I32, I32, F32, P],
    "pk_silu_and_mul_il": [P, P, I32, I32, P],
    "pk_skinny_gemm": [P, P, P, P, I32, I32, I32, I32, I32, I32, I32, P],
    "pk_splitk_reduce": [P, P, I32, I32, I32, I32, I32, P],
    "pk_splitk_add_rmsnorm": [P, P, P, P, I32, I32, I32, F32, P],
    "pk_splitk_add_rmsnorm_route": [P, P, P, P, I32, I32, I32, F32, P, I32, I32, I32, P, P, P],
    "pk_qkv_reduce_rope_cache": [P, P, I32, I32, I32, I32, P, P, P, P, P, I32, P],
    "pk_skinny_gemm_ex": [P, I32, P],
    "pk_mlp_fused": [P, P, P, P],
    "pk_qkv_attn_fused": [P, P, P, P, P, P, P, P, P, P, P, I32, I32, I32, I32, I32, F32, I32, P, P],
    "pk_gemm_args_size": [],
    "pk_norm_apply": [P, P, P, I32, P, I32, I32, F32, P],
    "pk_copy_from_host": [P, P, I64, P],
    "pk_residual_parts": [P, P, I32, I32, I32, P, P],
    "pk_car_gemm": [P, P, I32, P, P, I32, I32, P, I32, I32, P, P],
}


def lib() -> ctypes.CDLL:
    global _lib
    if _lib is None:
        with _lock:
            if _lib is None:
                l = load_cdll("libpk_kernels")
                for name, argtypes in SIGNATURES.items():
                    fn = getattr(l, name, None)
                    if fn is None:
                        continue
                    fn.argtypes = argtypes
                    fn.restype = ctypes.c_int
                _lib = l
    return _lib


def has(name: str) -> bool:
    return getattr(lib(), name, None) is not None


class KernelError(RuntimeError):
    pass


def check(rc: int, name: str) -> None:
    if rc != 0:
        raise KernelError(f"{name} failed with code {rc} "
                          f"({'unsupported shape' if rc < 0 else 'HIP error'})")


def stream_ptr(device: Optional[torch.device] = None) -> int:
    return torch.cuda.current_stream(device).cuda_stream


def ptr(t: Optional[torch.Tensor]) -> Optional[int]:
    return None if t is None else t.data_ptr()


def call(name: str, *args) -> None:
    fn = getattr(lib(), name)
    check(fn(*args), name)
