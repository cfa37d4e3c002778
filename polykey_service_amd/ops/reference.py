"""fp32 PyTorch reference implementations of every hand-written kernel.

Used (a) as the numerics oracle in ``tests/kernels`` (each HIP kernel is compared against
the op here) and (b) on CPU tensors so the whole engine runs in the GPU-less dev container.
Layouts are the ones the kernels use:

* K cache  ``[num_blocks, n_kv, block_size, head_dim]`` (token rows contiguous)
* V cache  ``[num_blocks, n_kv, head_dim, block_size]`` (stored transposed, so the P·V MFMA
  reads 8 consecutive tokens of one channel as one 16-byte vector)
* slot = block_id * block_size + offset; slot < 0 means "do not write" (padding rows)
"""
from __future__ import annotations

import math
from typing import Optional

import numpy as np
import torch


# ----------------------------------------------------------------------------- norms
def rms_norm(x: torch.Tensor, weight: torch.Tensor, eps: float) -> torch.Tensor:
    xf = x.float()
    r = torch.rsqrt(xf.pow(2).mean(-1, keepdim=True) + eps)
    return ((xf * r).to(x.dtype).float() * weight.float()).to(x.dtype)


def fused_add_rms_norm(x: torch.Tensor, residual: torch.Tensor, weight: torch.Tensor, eps: float):
    residual.copy_((x.float() + residual.float()).to(residual.dtype))
    x.copy_(rms_norm(residual, weight, eps))
    return x, residual


def silu_and_mul(x: torch.Tensor) -> torch.Tensor:
    d = x.shape[-1] // 2
    g, u = x[..., :d].float(), x[..., d:].float()
    return (torch.nn.functional.silu(g).to(x.dtype).float() * u).to(x.dtype)


def silu_and_mul_interleaved(x: torch.Tensor, block: int = 16) -> torch.Tensor:
    """x: [T, 2I] with gate/up interleaved in blocks of ``block`` columns."""
    T, I2 = x.shape[0], x.shape[-1]
    v = x.reshape(-1, I2 // (2 * block), 2, block)
    g, u = v[:, :, 0].reshape(-1, I2 // 2).float(), v[:, :, 1].reshape(-1, I2 // 2).float()
    return (torch.nn.functional.silu(g).to(x.dtype).float() * u).to(x.dtype).view(x.shape[:-1] + (I2 // 2,))


# ------------------------------------------------------------------------------ rope
def rope_inv_freq(head_dim: int, theta: float, scaling: Optional[dict] = None) -> torch.Tensor:
    inv = 1.0 / (theta ** (torch.arange(0, head_dim, 2, dtype=torch.float64) / head_dim))
    if scaling and scaling.get("rope_type", scaling.get("type")) == "llama3":
        factor = scaling["factor"]
        lo, hi = scaling.get("low_freq_factor", 1.0), scaling.get("high_freq_factor", 4.0)
        old = scaling.get("original_max_position_embeddings", 8192)
        lo_wl, hi_wl = old / lo, old / hi
        wl = 2 * math.pi / inv
        smooth = (old / wl - lo) / (hi - lo)
        scaled = torch.where(wl > lo_wl, inv / factor, inv)
        mid = (1 - smooth) * inv / factor + smooth * inv
        is_mid = (wl <= lo_wl) & (wl >= hi_wl)
        inv = torch.where(is_mid, mid, scaled)
    return inv.float()


def rope_cos_sin_cache(max_pos: int, head_dim: int, theta: float, scaling: Optional[dict] = None,
                       device=None) -> torch.Tensor:
    """[max_pos, head_dim] fp32: cos in [:, :hd/2], sin in [:, hd/2:]."""
    inv = rope_inv_freq(head_dim, theta, scaling).double()
    t = torch.arange(max_pos, dtype=torch.float64)
    f = torch.outer(t, inv)
    return torch.cat([f.cos(), f.sin()], dim=-1).float().to(device)


def apply_rope(x: torch.Tensor, positions: torch.Tensor, cos_sin: torch.Tensor) -> torch.Tensor:
    """Neox/HF ``rotate_half`` RoPE. x: [T, H, D] → rotated, same dtype (fp32 math)."""
    D = x.shape[-1]
    cs = cos_sin[positions.long()].float()
    cos, sin = cs[:, None, : D // 2], cs[:, None, D // 2:]
    xf = x.float()
    x1, x2 = xf[..., : D // 2], xf[..., D // 2:]
    return torch.cat([x1 * cos - x2 * sin, x2 * cos + x1 * sin], dim=-1).to(x.dtype)


_KIDX: dict = {}


def kcache_index(bs: int, device=None) -> torch.Tensor:
    """[bs, 128] flat position of K element (token, dim) inside one (block, kv head) slab of the
    paged K cache: fragment-native 32-token tiles (csrc/kernels/common.h ``kcache_off``)."""
    if bs % 32:
        raise ValueError(f"the K-cache layout needs a block size that is a multiple of 32, got {bs}")
    key = (bs, str(device))
    if key not in _KIDX:
        k = torch.arange(bs).view(bs, 1)
        d = torch.arange(128).view(1, 128)
        kt = k & 31
        lane = 16 * (d >> 5) + 4 * (kt >> 3) + (kt & 3)
        _KIDX[key] = ((k >> 5) * 4096 + ((((kt >> 2) & 1) * 4 + ((d >> 3) & 3)) * 64 + lane) * 8 + (d & 7)).to(device)
    return _KIDX[key]


_VIDX: dict = {}


def vcache_index(bs: int, device=None) -> torch.Tensor:
    """[bs, 128] flat position of V element (token, dim) inside one (block, kv head) slab of the
    paged V cache: per 32-token tile [d / 16][key / 8][d % 16][key % 8] (common.h ``vcache_off``)."""
    if bs % 32:
        raise ValueError(f"the V-cache layout needs a block size that is a multiple of 32, got {bs}")
    key = (bs, str(device))
    if key not in _VIDX:
        k = torch.arange(bs).view(bs, 1)
        d = torch.arange(128).view(1, 128)
        kt = k & 31
        _VIDX[key] = ((k >> 5) * 4096 + ((((d >> 4) << 2) + (kt >> 3)) * 16 + (d & 15)) * 8 + (kt & 7)).to(device)
    return _VIDX[key]


def v_cache_logical(v_cache: torch.Tensor) -> torch.Tensor:
    """The physical V cache [blocks, n_kv, 128, bs] as logical (token, dim) rows [blocks, n_kv, bs, 128]."""
    nb, nkv, hd, bs = v_cache.shape
    return v_cache.reshape(nb, nkv, bs * hd)[:, :, vcache_index(bs, v_cache.device).view(-1)].view(nb, nkv, bs, hd)


def k_cache_logical(k_cache: torch.Tensor) -> torch.Tensor:
    """The physical K cache [blocks, n_kv, bs, 128] as logical (token, dim) rows."""
    nb, nkv, bs, hd = k_cache.shape
    return k_cache.reshape(nb, nkv, bs * hd)[:, :, kcache_index(bs, k_cache.device).view(-1)].view(nb, nkv, bs, hd)


def rope_and_cache(qkv: torch.Tensor, positions: torch.Tensor, cos_sin: torch.Tensor,
                   k_cache: Optional[torch.Tensor], v_cache: Optional[torch.Tensor],
                   slot_mapping: Optional[torch.Tensor], nq: int, nkv: int, hd: int) -> torch.Tensor:
    """Rotate q,k of the fused QKV output in place and scatter k,v into the paged cache."""
    T = qkv.shape[0]
    view = qkv.view(T, nq + 2 * nkv, hd)
    q, k, v = view[:, :nq], view[:, nq:nq + nkv], view[:, nq + nkv:]
    q.copy_(apply_rope(q, positions, cos_sin))
    k.copy_(apply_rope(k, positions, cos_sin))
    if k_cache is not None and slot_mapping is not None:
        bs = k_cache.shape[2]
        sm = slot_mapping.long()
        valid = sm >= 0
        if valid.any():
            s = sm[valid]
            blk, off = s // bs, s % bs
            n, nkv_ = blk.numel(), k_cache.shape[1]
            kflat = k_cache.view(k_cache.shape[0], nkv_, bs * hd)
            pos = kcache_index(bs, k_cache.device)[off]  # [n, 128] fragment-native positions
            kflat[blk.view(n, 1, 1), torch.arange(nkv_, device=k_cache.device).view(1, nkv_, 1),
                  pos.view(n, 1, hd)] = k[valid].to(k_cache.dtype)
            vflat = v_cache.view(v_cache.shape[0], nkv_, bs * hd)
            vpos = vcache_index(bs, v_cache.device)[off]
            vflat[blk.view(n, 1, 1), torch.arange(nkv_, device=v_cache.device).view(1, nkv_, 1),
                  vpos.view(n, 1, hd)] = v[valid].to(v_cache.dtype)
    return q


# ------------------------------------------------------------------------- attention
def gather_kv(k_cache, v_cache, block_table, n_tokens):
    """→ K [n, n_kv, D], V [n, n_kv, D] for one sequence."""
    bs = k_cache.shape[2]
    nb = (n_tokens + bs - 1) // bs
    blocks = block_table[:nb].long()
    k = k_cache_logical(k_cache[blocks]).permute(0, 2, 1, 3).reshape(nb * bs, k_cache.shape[1], -1)[:n_tokens]
    v = v_cache_logical(v_cache[blocks]).permute(0, 2, 1, 3).reshape(nb * bs, v_cache.shape[1], -1)[:n_tokens]
    return k, v


def paged_attention(q: torch.Tensor, k_cache: torch.Tensor, v_cache: torch.Tensor, block_tables: torch.Tensor,
                    context_lens: torch.Tensor, cu_seqlens_q: torch.Tensor, scale: float) -> torch.Tensor:
    """Causal GQA attention of each sequence's new query tokens against its whole paged
    context.  Query ``i`` of a chunk of ``L`` tokens sits at absolute position
    ``ctx - L + i`` and attends to keys ``[0, ctx - L + i]``.  q: [T, nq, D] → [T, nq, D]."""
    T, nq, D = q.shape
    nkv = k_cache.shape[1]
    g = nq // nkv
    out = torch.zeros_like(q)
    cu = cu_seqlens_q.tolist()
    ctxs = context_lens.tolist()
    for s in range(len(ctxs)):
        a, b = cu[s], cu[s + 1]
        L, ctx = b - a, int(ctxs[s])
        if L == 0 or ctx == 0:
            continue
        k, v = gather_kv(k_cache, v_cache, block_tables[s], ctx)
        k = k.float().repeat_interleave(g, dim=1)  # [ctx, nq, D]
        v = v.float().repeat_interleave(g, dim=1)
        qs = q[a:b].float()  # [L, nq, D]
        scores = torch.einsum("lhd,thd->hlt", qs, k) * scale
        pos = torch.arange(ctx - L, ctx)[:, None]
        keys = torch.arange(ctx)[None, :]
        scores = scores.masked_fill((keys > pos)[None], float("-inf"))
        p = torch.softmax(scores, dim=-1)
        out[a:b] = torch.einsum("hlt,thd->lhd", p, v).to(q.dtype)
    return out


# --------------------------------------------------------------------------- sampling
_M32 = np.uint64(0xFFFFFFFF)


def _fmix32(h: np.ndarray) -> np.ndarray:
    h = h & _M32
    h ^= h >> np.uint64(16)
    h = (h * np.uint64(0x85EBCA6B)) & _M32
    h ^= h >> np.uint64(13)
    h = (h * np.uint64(0xC2B2AE35)) & _M32
    h ^= h >> np.uint64(16)
    return h


def philox_uniform(seed: int, offset: int, n: int) -> np.ndarray:
    """The kernel's counter-based uniform(0,1) stream, bit-exact (uint32 arithmetic)."""
    s = np.uint64(seed & 0xFFFFFFFF)
    h = (s * np.uint64(0x9E3779B1) + np.uint64(0x7F4A7C15)) & _M32
    h = (h ^ ((np.uint64(offset & 0xFFFFFFFF) + np.uint64(0x85EBCA6B) + ((h << np.uint64(6)) & _M32)
               + (h >> np.uint64(2))) & _M32)) & _M32
    h = _fmix32(np.array(h, dtype=np.uint64))
    idx = np.arange(n, dtype=np.uint64)
    x = _fmix32(h ^ ((idx * np.uint64(0xC2B2AE35)) & _M32))
    return ((x >> np.uint64(8)).astype(np.float64) + 0.5) * (1.0 / (1 << 24))


def sampling_mask(logits: torch.Tensor, temperature: float, top_k: int, top_p: float, min_p: float) -> torch.Tensor:
    """Boolean mask of tokens allowed by top-k → top-p → min-p (sort-based, HF order)."""
    x = logits.float() / max(temperature, 1e-6)
    V = x.shape[-1]
    keep = torch.ones_like(x, dtype=torch.bool)
    if 0 < top_k < V:
        kth = torch.topk(x, top_k).values[..., -1:]
        keep &= x >= kth
    if 0.0 < top_p < 1.0:
        xm = x.masked_fill(~keep, float("-inf"))
        p = torch.softmax(xm, -1)
        sp, idx = torch.sort(p, descending=True)
        before = torch.cumsum(sp, -1) - sp
        k_sorted = before < top_p
        k_sorted[..., 0] = True
        m = torch.zeros_like(keep)
        m.scatter_(-1, idx, k_sorted)
        # ties with the smallest kept value stay in (threshold semantics of the kernel)
        thr = torch.where(m, x, torch.full_like(x, float("inf"))).min(-1, keepdim=True).values
        keep &= x >= thr
    if min_p > 0.0:
        p = torch.softmax(x, -1)
        keep &= p >= min_p * p.max(-1, keepdim=True).values
    return keep


def sample(logits: torch.Tensor, temperature, top_k, top_p, min_p, seeds, offsets) -> torch.Tensor:
    """Row-wise sampling with the kernel's RNG: greedy when temperature == 0, otherwise
    Gumbel-max over the allowed set.  Returns int64 [B]."""
    B, V = logits.shape
    out = torch.empty(B, dtype=torch.long)
    for b in range(B):
        t = float(temperature[b])
        row = logits[b].float().cpu()
        if t <= 0.0:
            out[b] = int(torch.argmax(row))
            continue
        keep = sampling_mask(row[None], t, int(top_k[b]), float(top_p[b]), float(min_p[b]))[0]
        u = torch.from_numpy(philox_uniform(int(seeds[b]), int(offsets[b]), V))
        gumbel = -torch.log(-torch.log(u))
        score = (row.double() / t + gumbel).masked_fill(~keep, float("-inf"))
        out[b] = int(torch.argmax(score))
    return out
