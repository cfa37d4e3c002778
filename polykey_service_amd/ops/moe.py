"""Mixture-of-experts dispatch (Mixtral): routing, expert grouping, grouped GEMM, combine.

Decode (T <= 64 tokens): everything stays on the device and is graph-capturable —
``topk_softmax`` → ``align`` (stable counting sort by expert) → ``permute`` → grouped skinny
GEMM for w13 with the fused SiLU epilogue → grouped skinny GEMM for w2 → weighted
``unpermute``.  An expert that received no token is skipped without reading its weights.

Prefill (T > 64): the same routing kernels, then ONE launch per projection of the grouped MFMA
GEMM of ``csrc/kernels/gemm_prefill.hip`` — it reads the expert row offsets on the device (no
read-back, no per-expert launches) and fuses SiLU(gate)*up into the w13 epilogue.

Expert parallelism: with ``e_lo, e_hi`` this rank only computes experts ``[e_lo, e_hi)``;
slots routed elsewhere get ``inv = -1`` and contribute zero, and the caller all-reduces the
combined output across the EP group (tokens are replicated by TP attention, so the combine is
the same all-reduce the dense MLP already does — see parallel/ep.py for the all-to-all form).
"""
from __future__ import annotations

import dataclasses

from typing import Optional, Tuple

import torch
import torch.nn.functional as F

from . import gemm, gemm_prefill, native, reference
from .gemm import silu_and_mul_interleaved


def topk_softmax(router_logits: torch.Tensor, k: int, renorm: bool = True) -> Tuple[torch.Tensor, torch.Tensor]:
    T, E = router_logits.shape
    if not router_logits.is_cuda:
        p = torch.softmax(router_logits.float(), -1)
        w, ids = torch.sort(p, dim=-1, descending=True, stable=True)  # ties → lower expert id, as the kernel
        w, ids = w[:, :k], ids[:, :k]
        if renorm:
            w = w / w.sum(-1, keepdim=True)
        return ids.to(torch.int32), w
    ids = torch.empty((T, k), dtype=torch.int32, device=router_logits.device)
    w = torch.empty((T, k), dtype=torch.float32, device=router_logits.device)
    native.call("pk_moe_topk_softmax", ids.data_ptr(), w.data_ptr(), router_logits.data_ptr(), T, E, k,
                router_logits.stride(0), int(renorm), native.stream_ptr())
    return ids, w


def align(ids: torch.Tensor, E: int, e_lo: int, e_hi: int):
    """→ offsets [E_local+1], sorted slots [n], inverse positions [n] (int32; -1 = not local)."""
    n = ids.numel()
    El = e_hi - e_lo
    dev = ids.device
    if not ids.is_cuda:
        flat = ids.reshape(-1).long()
        local = (flat >= e_lo) & (flat < e_hi)
        key = torch.where(local, flat - e_lo, torch.full_like(flat, El))
        order = torch.sort(key, stable=True).indices
        counts = torch.bincount(key, minlength=El + 1)[:El]
        offsets = torch.zeros(El + 1, dtype=torch.int32)
        offsets[1:] = torch.cumsum(counts, 0)
        m = int(offsets[-1])
        sorted_ = order[:m].to(torch.int32)
        inv = torch.full((n,), -1, dtype=torch.int32)
        inv[order[:m]] = torch.arange(m, dtype=torch.int32)
        return offsets, sorted_, inv
    offsets = torch.empty(El + 1, dtype=torch.int32, device=dev)
    sorted_ = torch.empty(n, dtype=torch.int32, device=dev)
    inv = torch.empty(n, dtype=torch.int32, device=dev)
    native.call("pk_moe_align", ids.data_ptr(), offsets.data_ptr(), sorted_.data_ptr(), inv.data_ptr(), n, E, e_lo,
                e_hi, native.stream_ptr())
    return offsets, sorted_, inv


def permute(x: torch.Tensor, sorted_: torch.Tensor, offsets: torch.Tensor, k: int) -> torch.Tensor:
    n = sorted_.numel()
    H = x.shape[-1]
    if not x.is_cuda:
        m = int(offsets[-1])
        return x[(sorted_[:m].long() // k)]
    out = torch.empty((n, H), dtype=x.dtype, device=x.device)
    native.call("pk_moe_permute", out.data_ptr(), x.data_ptr(), sorted_.data_ptr(), offsets.data_ptr(), n,
                offsets.numel() - 1, k, H, native.stream_ptr())
    return out


def unpermute(y: torch.Tensor, inv: torch.Tensor, w: torch.Tensor, T: int, k: int) -> torch.Tensor:
    H = y.shape[-1]
    if not y.is_cuda:
        out = torch.zeros((T, H), dtype=torch.float32)
        if y.shape[0] == 0:  # no slot routed to this rank's experts (EP): zero contribution
            return out.to(y.dtype)
        invl = inv.view(T, k).long()
        for j in range(k):
            valid = invl[:, j] >= 0
            idx = invl[:, j].clamp(min=0)
            out += torch.where(valid[:, None], y[idx].float() * w[:, j:j + 1].float(), torch.zeros(()))
        return out.to(y.dtype)
    out = torch.empty((T, H), dtype=y.dtype, device=y.device)
    native.call("pk_moe_unpermute", out.data_ptr(), y.data_ptr(), inv.data_ptr(), w.data_ptr(), T, k, H,
                native.stream_ptr())
    return out


def grouped_gemm(a: torch.Tensor, w: torch.Tensor, offsets: torch.Tensor, max_rows: int, silu: bool,
                 packed: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Rows of expert e = a[offsets[e]:offsets[e+1]] times w[e]^T (w: [E_local, N, K]).
    Decode-sized groups (<= ``gemm.DECODE_MAX_M`` rows; above 64 in 128-row tiles) run the
    weight-streaming decode GEMM of csrc/kernels/gemm_skinny.hip in grouped mode (``packed``:
    fragment-packed experts)."""
    E_local, N, K = w.shape
    n_out = N // 2 if silu else N
    if (a.is_cuda and max_rows <= gemm.DECODE_MAX_M and gemm.SKINNY_ENABLED and N % 128 == 0
            and K % 256 == 0):
        return gemm.grouped_linear(a, w, offsets, max_rows, silu, packed=packed)
    out = torch.empty((a.shape[0], n_out), dtype=a.dtype, device=a.device)
    if a.is_cuda and max_rows <= 64:
        native.call("pk_moe_gemm", out.data_ptr(), a.data_ptr(), w.data_ptr(), offsets.data_ptr(), max_rows, N, K,
                    out.stride(0), E_local, 2 if silu else 0, native.stream_ptr())
        return out
    if a.is_cuda and gemm_prefill.supported(N, K) and w.is_contiguous():
        return gemm_prefill.grouped_linear(a, w, offsets, silu=silu, out=out)
    offs = offsets.tolist()  # shapes the MFMA kernel does not tile: a library GEMM per expert
    for e in range(E_local):
        lo, hi = offs[e], offs[e + 1]
        if hi > lo:  # results land in their rows of `out` directly (no slice-assignment copy)
            if silu:
                silu_and_mul_interleaved(F.linear(a[lo:hi], w[e]), out=out[lo:hi])
            else:
                torch.matmul(a[lo:hi], w[e].t(), out=out[lo:hi])
    return out


@dataclasses.dataclass
class PendingCombine:
    """Expert outputs not yet combined: :func:`combine_add_rms_norm` does the weighted top-k
    combine, the residual add and the next RMSNorm in one kernel."""
    y: torch.Tensor      # [T*k, H] expert outputs in expert-sorted order
    inv: torch.Tensor    # [T*k] sorted position of (token, slot); -1 = expert on another EP rank
    w: torch.Tensor      # [T, k] routing weights
    T: int
    k: int

    def combine(self) -> torch.Tensor:
        return unpermute(self.y, self.inv, self.w, self.T, self.k)


def combine_add_rms_norm(p: PendingCombine, residual: torch.Tensor, weight: torch.Tensor, eps: float):
    """residual += combine(p); x = rms_norm(residual) * weight → (x, residual), one kernel."""
    H = residual.shape[-1]
    if not residual.is_cuda or H % 1024 or H > 8192:
        from .norm import fused_add_rms_norm
        return fused_add_rms_norm(p.combine(), residual, weight, eps)
    x = torch.empty_like(residual)
    native.call("pk_moe_combine_add_rmsnorm", x.data_ptr(), residual.data_ptr(), p.y.data_ptr(), p.inv.data_ptr(),
                p.w.data_ptr(), weight.data_ptr(), p.T, p.k, H, float(eps), native.stream_ptr())
    return x, residual


def fused_moe(x: torch.Tensor, router_w: torch.Tensor, w13: torch.Tensor, w2: torch.Tensor, k: int,
              e_lo: int = 0, e_hi: Optional[int] = None, w13_p: Optional[torch.Tensor] = None,
              w2_p: Optional[torch.Tensor] = None, defer_combine: bool = False,
              routing: Optional[Tuple[torch.Tensor, torch.Tensor]] = None):
    """Mixtral sparse MLP for this rank's experts.  x [T, H]; router_w [E, H]; w13 [E_l, 2I, H]
    (gate/up interleaved by 16); w2 [E_l, H, I].  Returns the (partial, if EP) combined output,
    or with ``defer_combine`` a :class:`PendingCombine` for the fused combine+add+norm.
    ``routing``: (ids, weights) already computed by the preceding norm kernel
    (:func:`gemm.partial_add_rms_norm_route`).

    Decode (T <= 64): expert sort, the w13 grouped GEMM gathering token rows itself (no
    permute pass) with the SiLU epilogue, the w2 grouped GEMM, and the combine (fused into the
    next residual add + RMSNorm when deferred)."""
    T = x.shape[0]
    E = router_w.shape[0]
    e_hi = E if e_hi is None else e_hi
    N13, K13 = w13.shape[1], w13.shape[2]
    if (x.is_cuda and T <= 64 and E <= 64 and gemm.SKINNY_ENABLED and N13 % 128 == 0 and K13 % 256 == 0
            and w2.shape[1] % 128 == 0 and w2.shape[2] % 256 == 0):
        if routing is not None:
            ids, wts = routing
        else:
            ids, wts = topk_softmax(F.linear(x, router_w), k)
        offsets, sorted_, inv = align(ids, E, e_lo, e_hi)
        h = gemm.grouped_linear(x, w13, offsets, T, True, packed=w13_p, a_rows=sorted_, a_row_div=k, n_rows=T * k)
        y = gemm.grouped_linear(h, w2, offsets, T, False, packed=w2_p)
        pending = PendingCombine(y, inv, wts, T, k)
        return pending if defer_combine else pending.combine()
    logits = F.linear(x, router_w)
    ids, wts = topk_softmax(logits, k)
    offsets, sorted_, inv = align(ids, E, e_lo, e_hi)
    xs = permute(x, sorted_, offsets, k)
    h = grouped_gemm(xs, w13, offsets, T, silu=True, packed=w13_p)
    y = grouped_gemm(h, w2, offsets, T, silu=False, packed=w2_p)
    return unpermute(y, inv, wts, T, k)


def fused_moe_reference(x, router_w, w13, w2, k, e_lo=0, e_hi=None):
    """Loop-over-experts oracle with fp32 GEMMs and the kernels' bf16 rounding points
    (projection outputs, SiLU and h are bf16 tensors in the fused path)."""
    E = router_w.shape[0]
    e_hi = E if e_hi is None else e_hi
    bf = lambda t: t.to(torch.bfloat16).float()
    p = torch.softmax(bf(x.float() @ router_w.float().t()), -1)
    w, ids = torch.topk(p, k, -1)
    w = w / w.sum(-1, keepdim=True)
    out = torch.zeros(x.shape, dtype=torch.float32, device=x.device)
    H = x.shape[1]
    for e in range(e_lo, e_hi):
        v = w13[e - e_lo].float().view(-1, 2, 16, H)
        g, u = v[:, 0].reshape(-1, H), v[:, 1].reshape(-1, H)
        h = bf(bf(torch.nn.functional.silu(bf(x.float() @ g.t()))) * bf(x.float() @ u.t()))
        y = bf(h @ w2[e - e_lo].float().t())
        sel = (ids == e).float() * w
        out += sel.sum(-1, keepdim=True) * y
    return out
