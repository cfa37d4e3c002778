"""Paged attention + fused RoPE/KV-cache write (HIP on GPU, fp32 reference on CPU).

Batch layout (see :class:`AttnMetadata`): the first ``num_decode`` tokens are decode tokens
(one per sequence), followed by the prefill tokens of ``num_prefill`` sequences (possibly
chunked, possibly with a cached prefix).  Decode goes through the split-K decode kernel,
prefill through the varlen causal kernel; both read K/V only from the paged cache (new
tokens are written by :func:`rope_and_cache` first).
"""
from __future__ import annotations

import dataclasses
import math
import os
from typing import Optional

import torch

from . import native, reference


@dataclasses.dataclass
class AttnMetadata:
    num_decode: int
    num_prefill: int
    num_prefill_tokens: int
    max_prefill_q_len: int
    slot_mapping: torch.Tensor              # [T] int32
    decode_block_tables: Optional[torch.Tensor] = None   # [nd, MB] int32
    decode_context_lens: Optional[torch.Tensor] = None   # [nd] int32
    prefill_block_tables: Optional[torch.Tensor] = None  # [np, MB] int32
    prefill_context_lens: Optional[torch.Tensor] = None  # [np] int32
    prefill_cu_q: Optional[torch.Tensor] = None          # [np+1] int32, relative to the first prefill token
    decode_part_o: Optional[torch.Tensor] = None         # split-K workspace
    decode_part_ml: Optional[torch.Tensor] = None
    decode_max_ctx: int = 0  # bound on every decode context of the step (0: block-table capacity)

    @property
    def num_tokens(self) -> int:
        return self.num_decode + self.num_prefill_tokens


_PART = 512  # must match kDecodePart in csrc/kernels/attention.hip
_PART_MIN = 128  # kDecodePartSmall: launches whose (seq, kv head) pairs cannot fill the chip
_FILL_SET = False


def apply_decode_fill() -> None:
    """POLYKEY_DECODE_FILL, applied once per process: the workgroup count below which decode
    attention takes 128-key partitions (csrc attention.hip decode_part; 0: always 512)."""
    global _FILL_SET
    if not _FILL_SET and os.environ.get("POLYKEY_DECODE_FILL") is not None:
        native.call("pk_set_decode_fill", int(os.environ["POLYKEY_DECODE_FILL"]))
    _FILL_SET = True


# g_decode_fill (csrc attn_decode.h): fewer (seq, kv head, partition) workgroups than this -> 128-key partitions
_DECODE_FILL = int(os.environ.get("POLYKEY_DECODE_FILL", "256"))


def decode_workspace(n_seqs: int, n_q: int, max_blocks: int, block_size: int, device, n_kv: int = 0,
                     kv_heads: Optional[int] = None) -> tuple:
    """Partition slabs for split-K decode attention.  A launch
    strides the slabs by its OWN partition count, so they are sized for the largest launch:
    ``n_seqs`` sequences at 512-key partitions, or the few sequences that take 128-key ones
    (csrc attention.hip decode_part: fewer than 256 (seq, kv head) workgroups, i.e. at most
    255 // kv_heads sequences).  ``kv_heads`` (kv heads per rank; else ``n_kv``) None: every
    launch sized at 128-key partitions (4x the full-batch need: ~4.3 GB at 256 seqs x 128k ctx
    for Llama-3-8B, taken from the KV-cache budget -- ADVICE r4)."""
    ctx = max_blocks * block_size
    n_small = (ctx + _PART_MIN - 1) // _PART_MIN
    if n_small <= 1:
        return None, None
    kvh = kv_heads or n_kv
    if kvh:
        seqs_small = min(n_seqs, (_DECODE_FILL - 1) // kvh)
        rows = max(n_seqs * ((ctx + _PART - 1) // _PART), seqs_small * n_small)
    else:
        rows = n_seqs * n_small
    o = torch.empty((rows * n_q, 128), dtype=torch.float32, device=device)
    ml = torch.empty((rows * n_q, 2), dtype=torch.float32, device=device)
    return o, ml


def rope_and_cache(qkv: torch.Tensor, positions: torch.Tensor, cos_sin: torch.Tensor, k_cache: torch.Tensor,
                   v_cache: torch.Tensor, slot_mapping: torch.Tensor, nq: int, nkv: int, hd: int = 128) -> None:
    """In place on ``qkv`` [T, (nq+2nkv)*hd]; writes K/V of every token with slot >= 0."""
    if not qkv.is_cuda:
        reference.rope_and_cache(qkv, positions, cos_sin, k_cache, v_cache, slot_mapping, nq, nkv, hd)
        return
    T = qkv.shape[0]
    assert qkv.stride(-1) == 1 and positions.dtype == torch.int32 and slot_mapping.dtype == torch.int32
    assert cos_sin.dtype == torch.float32 and k_cache.dtype == torch.bfloat16
    native.call("pk_rope_and_cache", qkv.data_ptr(), positions.data_ptr(), cos_sin.data_ptr(), k_cache.data_ptr(),
                v_cache.data_ptr(), slot_mapping.data_ptr(), T, nq, nkv, hd, k_cache.shape[2], qkv.stride(0), 0,
                native.stream_ptr())


def paged_attention(q: torch.Tensor, k_cache: torch.Tensor, v_cache: torch.Tensor, md: AttnMetadata,
                    scale: float, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """q: [T, nq, 128] view (row stride may exceed nq*128, e.g. inside the QKV buffer).
    Returns out: [T, nq*128] bf16."""
    T, nq, hd = q.shape
    nkv = k_cache.shape[1]
    bs = k_cache.shape[2]
    if out is None:
        out = torch.empty((T, nq * hd), dtype=q.dtype, device=q.device)
    if not q.is_cuda:
        _reference(q, k_cache, v_cache, md, scale, out)
        return out
    assert hd == 128 and q.stride(-1) == 1 and q.stride(1) == hd
    apply_decode_fill()
    stream = native.stream_ptr()
    nd = md.num_decode
    if nd > 0:
        bt = md.decode_block_tables
        native.call("pk_paged_decode", out.data_ptr(), q.data_ptr(), k_cache.data_ptr(), v_cache.data_ptr(),
                    bt.data_ptr(), md.decode_context_lens.data_ptr(),
                    native.ptr(md.decode_part_o) or 0, native.ptr(md.decode_part_ml) or 0,
                    nd, nq, nkv, bs, bt.stride(0), q.stride(0), out.stride(0),
                    float(scale), int(md.decode_max_ctx), stream)
    if md.num_prefill > 0:
        bt = md.prefill_block_tables
        qp = q[nd:]
        op = out[nd:]
        native.call("pk_paged_prefill", op.data_ptr(), qp.data_ptr(), k_cache.data_ptr(), v_cache.data_ptr(),
                    bt.data_ptr(), md.prefill_context_lens.data_ptr(), md.prefill_cu_q.data_ptr(), 0,
                    md.num_prefill, nq, nkv, bs, bt.shape[1], q.stride(0), out.stride(0), int(md.max_prefill_q_len),
                    float(scale), stream)
    return out


def _reference(q, k_cache, v_cache, md: AttnMetadata, scale, out):
    nd = md.num_decode
    o3 = out.view(out.shape[0], q.shape[1], q.shape[2])
    if nd > 0:
        cu = torch.arange(nd + 1, dtype=torch.int32)
        o3[:nd] = reference.paged_attention(q[:nd].contiguous(), k_cache, v_cache, md.decode_block_tables.cpu(),
                                            md.decode_context_lens.cpu(), cu, scale)
    if md.num_prefill > 0:
        o3[nd:] = reference.paged_attention(q[nd:].contiguous(), k_cache, v_cache, md.prefill_block_tables.cpu(),
                                            md.prefill_context_lens.cpu(), md.prefill_cu_q.cpu(), scale)


def default_scale(head_dim: int = 128) -> float:
    return 1.0 / math.sqrt(head_dim)


def paged_decode_from_qkv(p, positions: torch.Tensor, cos_sin: torch.Tensor, k_cache: torch.Tensor,
                          v_cache: torch.Tensor, md: AttnMetadata, scale: float, nq: int, nkv: int) -> torch.Tensor:
    """Pure-decode attention straight from the fused QKV projection's split-K slabs
    (``gemm.Partial``): the attention kernel reduces the slabs, applies RoPE, writes the new
    k / v into the paged cache and attends — one kernel instead of reduce+RoPE+cache then
    attention.  Returns [T, nq*128] bf16."""
    assert md.num_prefill == 0 and k_cache.shape[-1] == 128
    apply_decode_fill()
    T = p.M
    out = torch.empty((T, nq * 128), dtype=torch.bfloat16, device=p.buf.device)
    bt = md.decode_block_tables
    native.call("pk_paged_decode_qkv", out.data_ptr(), p.buf.data_ptr(), p.S, p.M, positions.data_ptr(),
                cos_sin.data_ptr(), md.slot_mapping.data_ptr(), k_cache.data_ptr(), v_cache.data_ptr(),
                bt.data_ptr(), md.decode_context_lens.data_ptr(), native.ptr(md.decode_part_o) or 0,
                native.ptr(md.decode_part_ml) or 0, md.num_decode, nq, nkv, k_cache.shape[2], bt.stride(0),
                out.stride(0), float(scale), int(md.decode_max_ctx), native.stream_ptr())
    return out
