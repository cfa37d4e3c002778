"""RMSNorm / fused residual-add RMSNorm / SiLU-and-mul (HIP on GPU, fp32 reference on CPU)."""
from __future__ import annotations

from typing import Optional

import torch

from . import native, reference


def rms_norm(x: torch.Tensor, weight: torch.Tensor, eps: float, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """y = x * rsqrt(mean(x^2) + eps) * w over the last dim of a 2-D [T, H] view."""
    if not x.is_cuda:
        return reference.rms_norm(x, weight, eps)
    H = x.shape[-1]
    x2 = x.reshape(-1, H)
    assert x2.stride(-1) == 1 and weight.is_contiguous() and x.dtype == torch.bfloat16
    T = x2.shape[0]
    if out is None:
        out = torch.empty((T, H), dtype=x.dtype, device=x.device)
    native.call("pk_rmsnorm", out.data_ptr(), x2.data_ptr(), weight.data_ptr(), T, H, x2.stride(0),
                out.stride(0), float(eps), native.stream_ptr())
    return out.view(x.shape)


def fused_add_rms_norm(x: torch.Tensor, residual: torch.Tensor, weight: torch.Tensor, eps: float):
    """In place: residual += x; x = rms_norm(residual) * w.  Returns (x, residual)."""
    if not x.is_cuda:
        return reference.fused_add_rms_norm(x, residual, weight, eps)
    assert x.is_contiguous() and residual.is_contiguous() and x.shape == residual.shape
    H = x.shape[-1]
    T = x.numel() // H
    native.call("pk_fused_add_rmsnorm", x.data_ptr(), residual.data_ptr(), weight.data_ptr(), T, H, float(eps),
                native.stream_ptr())
    return x, residual


def silu_and_mul(x: torch.Tensor, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """x: [T, 2I] = gate | up → silu(gate) * up: [T, I]."""
    if not x.is_cuda:
        return reference.silu_and_mul(x)
    assert x.is_contiguous() and x.dtype == torch.bfloat16
    I2 = x.shape[-1]
    T = x.numel() // I2
    if out is None:
        out = torch.empty(x.shape[:-1] + (I2 // 2,), dtype=x.dtype, device=x.device)
    native.call("pk_silu_and_mul", out.data_ptr(), x.data_ptr(), T, I2 // 2, native.stream_ptr())
    return out
