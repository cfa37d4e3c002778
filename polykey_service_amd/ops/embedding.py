"""Vocab-parallel token embedding (csrc/kernels/embedding.hip)."""
from __future__ import annotations

import torch
import torch.nn.functional as F

from . import native


def embedding(ids: torch.Tensor, table: torch.Tensor, vocab_start: int = 0, vocab_local: int = -1) -> torch.Tensor:
    """Rows ``table[ids - vocab_start]`` for ids in this rank's shard
    ``[vocab_start, vocab_start + vocab_local)``, zero rows for the others."""
    if vocab_local < 0:
        vocab_local = table.shape[0]
    T, H = ids.numel(), table.shape[1]
    if not ids.is_cuda:
        local = ids.long() - vocab_start
        mask = (local >= 0) & (local < vocab_local)
        x = F.embedding(torch.where(mask, local, torch.zeros_like(local)), table)
        return x * mask.unsqueeze(-1).to(x.dtype)
    ids32 = ids.reshape(-1)
    if ids32.dtype != torch.int32:
        ids32 = ids32.to(torch.int32)
    out = torch.empty((T, H), dtype=table.dtype, device=table.device)
    native.call("pk_embedding", out.data_ptr(), table.data_ptr(), ids32.contiguous().data_ptr(), T, H, vocab_start,
                vocab_local, native.stream_ptr())
    return out.view(*ids.shape, H)
