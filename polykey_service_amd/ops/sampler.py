"""Token sampling (HIP kernel on GPU, reference on CPU).

Per-row parameters are device tensors so a decode step (logits → tokens) can be captured in
a HIP graph: ``temperature`` f32 (0 → greedy), ``top_k`` i32 (0 → off), ``top_p`` f32
(1 → off), ``min_p`` f32 (0 → off), ``seeds`` i32 and ``offsets`` i32 (the per-request
token index, so a seeded request reproduces regardless of how it was batched).
"""
from __future__ import annotations

from typing import Optional

import torch

from . import native, reference


def sample(logits: torch.Tensor, temperature: torch.Tensor, top_k: torch.Tensor, top_p: torch.Tensor,
           min_p: torch.Tensor, seeds: torch.Tensor, offsets: torch.Tensor,
           out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """logits [B, V] (bf16 or fp32) → int32 token ids [B]."""
    B, V = logits.shape
    if not logits.is_cuda:
        return reference.sample(logits, temperature, top_k, top_p, min_p, seeds, offsets).to(torch.int32)
    assert logits.stride(-1) == 1
    if out is None:
        out = torch.empty(B, dtype=torch.int32, device=logits.device)
    dtype = 0 if logits.dtype == torch.bfloat16 else 1
    assert logits.dtype in (torch.bfloat16, torch.float32)
    native.call("pk_sample", out.data_ptr(), logits.data_ptr(), temperature.data_ptr(), top_k.data_ptr(),
                top_p.data_ptr(), min_p.data_ptr(), seeds.data_ptr(), offsets.data_ptr(), 0, B, V,
                logits.stride(0), dtype, native.stream_ptr())
    return out


def greedy(logits: torch.Tensor, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    if not logits.is_cuda:
        return torch.argmax(logits.float(), dim=-1).to(torch.int32)
    B, V = logits.shape
    if out is None:
        out = torch.empty(B, dtype=torch.int32, device=logits.device)
    dtype = 0 if logits.dtype == torch.bfloat16 else 1
    native.call("pk_sample", out.data_ptr(), logits.data_ptr(), 0, 0, 0, 0, 0, 0, 0, B, V, logits.stride(0), dtype,
                native.stream_ptr())
    return out
