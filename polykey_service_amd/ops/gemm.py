"""Projection GEMMs: hand-written weight-streaming kernel for decode-sized M, hipBLASLt otherwise.

``y = x @ W^T`` with ``W`` in PyTorch ``[N, K]`` layout.  For ``M <= 64`` on the GPU the HIP
kernel in ``csrc/kernels/gemm_skinny.hip`` streams ``W`` once at (near) HBM rate and can
(a) emit fp32 split-K partial slabs that the *consumer* reduces (``Partial``), or (b) apply
SiLU(gate)*up in its epilogue when the gate/up rows are interleaved in blocks of 16
(:func:`interleave_gate_up`).  Prefill-sized M goes to ``F.linear`` (hipBLASLt), whose tuned
MFMA kernels are the right tool for compute-bound shapes.
"""
from __future__ import annotations

import ctypes
import dataclasses
from typing import NamedTuple, Optional

import torch
import torch.nn.functional as F

from . import native, reference

import os

# automatic dispatch (linear / linear_silu on any caller, prefill chunks included) picks the
# skinny kernel up to 64 rows; the decode chain (llama _forward_rowscale, LM head, EP expert
# groups) uses it up to DECODE_MAX_M in row tiles whose workgroups share each W tile through one
# XCD's L2 (csrc/kernels/gemm_skinny.hip "Row tiles", profiles/r3_decode_rows.txt)
SKINNY_MAX_M = 64
DECODE_MAX_M = 512
# the fused decode launches (qkv_attn_fused, mlp_fused) take up to one 128-row tile; above 64 rows
# its row scale reads at most 16 norm parts (the TP=1 chain's residual_parts: H / 512)
FUSED_MAX_M = 128
FUSED_MT8_MAX_PARTS = 16
SKINNY_TILE_M = 128  # rows per row tile above 64 (the kernel's MT = 8 variant)
# measured best (tools/bench_gemm.py, cold weights): ~0.75-1 workgroup per CU
_TARGET_WGS = 192
_ROWS_PER_WG = 128
_KCHUNK = 256
# The hand-written decode GEMM is used when it beats hipBLASLt on the shape (see
# tools/bench_gemm.py and profiles/); POLYKEY_SKINNY_GEMM=0/1 forces it off/on.
SKINNY_ENABLED = os.environ.get("POLYKEY_SKINNY_GEMM", "1") == "1"
# decode MLP as one launch (gate_up -> down hand-off in-kernel, mlp_fused); 0: two launches.  Not
# when its gate_up must be split over K (the 70B TP=8 shard's 56 n-blocks): measured 1.4 us / layer
# slower than the two launches there (profiles/r4_tp_solo.md; that variant was removed in round 6)
MLP_FUSED = os.environ.get("POLYKEY_MLP_FUSED", "1") == "1"
# the QKV -> attention launch wins where each kv head's attention tiles wait on a slice of the QKV
# tiles (8B: 8 kv heads); with one or two kv heads per rank (70B TP=8 / TP=4) every attention tile
# waits for the whole projection and the launch measured slower (26.6 vs ~20 us per layer at
# 70B TP=8, profiles/r4_tp_solo.md)
QKV_ATTN_MIN_KV = 4
# the two-launch decode QKV (TP shards with few kv heads) as 64-row n-blocks at half the split:
# half the fp32 slabs the attention prologue sums (70B TP=8: 6.66-6.67 vs 6.68 ms, neutral)
QKV_HALF = True
# bf16-out decode GEMMs whose 128-row n-blocks cannot fill the chip run as 64-row n-blocks (the 70B
# TP=8 LM-head shard: 126 -> 252 workgroups; per-rank step 6.52 vs 6.54 ms, profiles/r5_lmhalf.jsonl).
# Measured and removed in round 6: the half-split projections at 2x their split (profiles/r5_osplit.jsonl),
# explicit QKV splits (r5_split_ab.jsonl)
PACKED_BIT = 16


MODE_BF16, MODE_PARTIAL, MODE_SILU, MODE_ADD_RES_NORM, MODE_QKV_ROPE, MODE_PUSH = 0, 1, 2, 3, 4, 6
# TP decode: the row-parallel projections' GEMM epilogue pushes its finished tiles into the owner
# ranks' IPC slots (MODE_PUSH, :func:`push_projection`) and the collective starts at the
# reduce-scatter (custom_ar.reduce_residual_pushed).  Bit-identical to GEMM + fused collective; off
# by default until an 8-GPU run has timed it (one GPU cannot show the xGMI traffic it hides).
# (Removed in round 6, measured slower in rounds 4-5: the split gate_up reduced + SiLU'd in-launch,
# 6.78 vs 6.68 ms per 70B TP=8 rank step, r5_tp_ab.jsonl; the unsplit 64-row gate_up, 7.75 vs
# 6.51 ms, r5_kr1.jsonl.)
TP_PUSH = os.environ.get("POLYKEY_TP_PUSH", "0") == "1"
NORM_BIT = 32


class GemmArgs(ctypes.Structure):
    """Mirror of ``struct GemmArgs`` in csrc/kernels/gemm_skinny.hip (checked against
    ``pk_gemm_args_size`` on first use)."""
    _fields_ = [("out", ctypes.c_void_p), ("partial", ctypes.c_void_p), ("A", ctypes.c_void_p),
                ("W", ctypes.c_void_p), ("M", ctypes.c_int), ("N", ctypes.c_int), ("K", ctypes.c_int),
                ("lda", ctypes.c_int), ("ldo", ctypes.c_int), ("S", ctypes.c_int), ("counters", ctypes.c_void_p),
                ("nrm_parts", ctypes.c_void_p), ("nrm_w", ctypes.c_void_p), ("nrm_nparts", ctypes.c_int),
                ("eps", ctypes.c_float), ("residual", ctypes.c_void_p), ("sumsq_parts", ctypes.c_void_p),
                ("positions", ctypes.c_void_p), ("cos_sin", ctypes.c_void_p), ("k_cache", ctypes.c_void_p),
                ("v_cache", ctypes.c_void_p), ("slots", ctypes.c_void_p), ("nq", ctypes.c_int),
                ("nkv", ctypes.c_int), ("bs", ctypes.c_int), ("row_offsets", ctypes.c_void_p),
                ("w_stride", ctypes.c_longlong), ("groups", ctypes.c_int), ("max_group_rows", ctypes.c_int),
                ("a_rows", ctypes.c_void_p), ("a_row_div", ctypes.c_int), ("row_scale", ctypes.c_int),
                ("row_tiles", ctypes.c_int), ("tile_rows", ctypes.c_int), ("push_peers", ctypes.c_void_p),
                ("push_bytes", ctypes.c_longlong), ("push_rank", ctypes.c_int), ("push_world", ctypes.c_int)]


_ARGS_CHECKED = False


class RowScale(NamedTuple):
    """Folded RMSNorm: A is the residual stream, W's columns carry the norm weight
    (:func:`fold_norm`), and output row m is scaled by rinv[m] = rsqrt(sum(parts[:, m]) / K + eps)
    with ``parts`` [nparts, M] from :func:`residual_parts`."""
    parts: torch.Tensor
    eps: float


class NormIn(NamedTuple):
    """RMSNorm applied in a GEMM's A-staging prologue: A is the residual stream, ``parts`` the
    per-row sum-of-squares parts [nparts, M] a MODE_ADD_RES_NORM epilogue produced."""
    parts: torch.Tensor
    weight: torch.Tensor
    eps: float


def _launch_ex(mode: int, x: torch.Tensor, w: torch.Tensor, packed: Optional[torch.Tensor], S: int,
               out: Optional[torch.Tensor] = None, ws: Optional[torch.Tensor] = None,
               counters: Optional[torch.Tensor] = None, norm: Optional[NormIn] = None,
               rowscale: Optional[RowScale] = None, **kw) -> None:
    global _ARGS_CHECKED
    if not _ARGS_CHECKED:
        n = native.lib().pk_gemm_args_size()
        assert n == ctypes.sizeof(GemmArgs), f"GemmArgs layout mismatch: C {n} vs ctypes {ctypes.sizeof(GemmArgs)}"
        _ARGS_CHECKED = True
    M, K = x.shape
    M = kw.pop("m_override", None) or M  # grouped + gathered A: rows of the grouped output
    N = kw.pop("n_override", None) or w.shape[0]
    if "groups" in kw:
        N = w.shape[0] // kw["groups"]
    a = GemmArgs()
    a.out = native.ptr(out)
    a.partial = native.ptr(ws)
    a.A = x.data_ptr()
    a.W = (packed if packed is not None else w).data_ptr()
    a.M, a.N, a.K, a.lda, a.S = M, N, K, x.stride(0), S
    a.ldo = out.stride(0) if out is not None else N
    a.counters = native.ptr(counters)
    if norm is not None:
        mode |= NORM_BIT
        a.nrm_parts = norm.parts.data_ptr()
        a.nrm_nparts = norm.parts.shape[0]
        a.nrm_w = norm.weight.data_ptr()
        a.eps = float(norm.eps)
    if rowscale is not None:
        a.row_scale = 1
        a.nrm_parts = rowscale.parts.data_ptr()
        a.nrm_nparts = rowscale.parts.shape[0]
        a.eps = float(rowscale.eps)
    for k, v in kw.items():
        setattr(a, k, v.data_ptr() if isinstance(v, torch.Tensor) else v)
    mode |= _wmode(packed)
    native.call("pk_skinny_gemm_ex", ctypes.byref(a), mode, native.stream_ptr())


HALF_BIT = 128  # 64-row n-blocks (KR = 1): twice the n-blocks, half the split-K
ROWS64_BIT = 256  # M > 64: 64-row tiles instead of 128 (A/B only: tools/bench_gemm_rows.py)


def linear_add_residual(x: torch.Tensor, w: torch.Tensor, ws: torch.Tensor, counters: torch.Tensor,
                        residual: torch.Tensor, sumsq_parts: torch.Tensor, S: Optional[int] = None,
                        packed: Optional[torch.Tensor] = None, half: bool = False) -> torch.Tensor:
    """residual += x @ w^T (split-K reduced in-kernel by the last split of each n-block to
    arrive) and sumsq_parts[N/nblk, M] = per-row sums of squares of the new residual over each
    n-block of columns (128, or 64 with ``half``), for the next projection's RowScale / NormIn.
    Returns the parts view."""
    M, K = x.shape
    N = w.shape[0]
    nblk = 64 if half else 128
    S = S or choose_split(N, K, M)
    assert ws.numel() >= S * M * N and sumsq_parts.numel() >= (N // nblk) * M and counters.numel() >= N // nblk
    _launch_ex(MODE_ADD_RES_NORM | (HALF_BIT if half else 0), x, w, packed, S, ws=ws, counters=counters,
               residual=residual, sumsq_parts=sumsq_parts)
    return sumsq_parts.view(-1)[: (N // nblk) * M].view(N // nblk, M)


def linear_qkv_rope(x: torch.Tensor, w: torch.Tensor, ws: torch.Tensor, counters: torch.Tensor,
                    positions: torch.Tensor, cos_sin: torch.Tensor, k_cache: torch.Tensor, v_cache: torch.Tensor,
                    slots: torch.Tensor, nq: int, nkv: int, S: Optional[int] = None,
                    packed: Optional[torch.Tensor] = None, norm: Optional[NormIn] = None) -> torch.Tensor:
    """Fused QKV projection (split-K reduced in-kernel) + RoPE + paged KV write → q [M, nq, 128].
    With ``norm``, ``x`` is the residual stream and the RMSNorm is applied on the fly."""
    M, K = x.shape
    N = w.shape[0]
    assert N == (nq + 2 * nkv) * 128
    S = S or choose_split(N, K, M)
    assert ws.numel() >= S * M * N and counters.numel() >= N // 128
    q = torch.empty((M, nq, 128), dtype=torch.bfloat16, device=x.device)
    _launch_ex(MODE_QKV_ROPE, x, w, packed, S, out=q.view(M, nq * 128), ws=ws, counters=counters, norm=norm,
               positions=positions, cos_sin=cos_sin, k_cache=k_cache, v_cache=v_cache, slots=slots, nq=nq,
               nkv=nkv, bs=k_cache.shape[2])
    return q


def grouped_linear(a: torch.Tensor, w: torch.Tensor, offsets: torch.Tensor, max_rows: int, silu: bool,
                   packed: Optional[torch.Tensor] = None, ws: Optional[torch.Tensor] = None,
                   S: int = 1, a_rows: Optional[torch.Tensor] = None, a_row_div: int = 1,
                   n_rows: Optional[int] = None) -> torch.Tensor:
    """Grouped decode GEMM (MoE experts): rows ``a[offsets[e]:offsets[e+1]]`` times ``w[e]^T``,
    ``w`` [G, N, K] (``packed``: :func:`pack_weight` of ``w.view(G*N, K)``), every group at most
    ``max_rows`` rows (above 64: 128-row tiles).  One launch; groups without rows read no weights.  ``silu``: interleaved gate/up →
    [R, N/2] bf16.  Otherwise ``S`` > 1 returns fp32 split-K slabs [S, R, N] in ``ws``."""
    G, N, K = w.shape
    # a_rows: gather A rows (a_rows[i] // a_row_div) instead of reading group-contiguous rows —
    # the MoE permute folded into the GEMM's A staging; n_rows = rows of the grouped output
    R = n_rows if n_rows is not None else a.shape[0]
    out = None
    if silu or S == 1:
        out = torch.empty((R, N // 2 if silu else N), dtype=a.dtype, device=a.device)
    mode = MODE_SILU if silu else (MODE_BF16 if S == 1 else MODE_PARTIAL)
    M2 = a  # A rows are addressed through the offsets
    args = dict(row_offsets=offsets, w_stride=N * K, groups=G, max_group_rows=max_rows)
    if a_rows is not None:
        args.update(a_rows=a_rows, a_row_div=a_row_div, m_override=R)
    _launch_ex(mode, M2, w.view(G * N, K), None if packed is None else packed.view(G * N, K), S, out=out,
               ws=ws if S > 1 else None, **args)
    return out if out is not None else ws


def norm_apply(residual: torch.Tensor, parts: torch.Tensor, weight: torch.Tensor, eps: float) -> torch.Tensor:
    """rms_norm(residual) * weight using precomputed per-row sum-of-squares parts."""
    M, H = residual.shape
    x = torch.empty_like(residual)
    native.call("pk_norm_apply", x.data_ptr(), residual.data_ptr(), parts.data_ptr(), parts.shape[0],
                weight.data_ptr(), M, H, float(eps), native.stream_ptr())
    return x


@dataclasses.dataclass
class Partial:
    """fp32 split-K slabs ``buf[:S*M*N]`` viewed as [S, M, N] (not yet summed)."""
    buf: torch.Tensor
    S: int
    M: int
    N: int

    def view(self) -> torch.Tensor:
        return self.buf[: self.S * self.M * self.N].view(self.S, self.M, self.N)


def interleave_gate_up(gate: torch.Tensor, up: torch.Tensor, block: int = 16) -> torch.Tensor:
    """[I, K] gate, [I, K] up → [2I, K] with rows [g0..g15, u0..u15, g16.., u16.., ...]."""
    I, K = gate.shape
    assert I % block == 0
    return torch.stack([gate.view(I // block, block, K), up.view(I // block, block, K)], dim=1).reshape(2 * I, K)


def deinterleave_gate_up(w: torch.Tensor, block: int = 16):
    I2, K = w.shape
    v = w.view(I2 // (2 * block), 2, block, K)
    return v[:, 0].reshape(I2 // 2, K), v[:, 1].reshape(I2 // 2, K)


def choose_split(N: int, K: int, M: int, target: Optional[int] = None) -> int:
    """Smallest power-of-two K split giving >= ``target`` workgroups (128 W rows x one row tile
    each): 192 for one row tile, 384 when several row tiles share each W tile through the L2
    (tools/bench_gemm_rows.py, profiles/r3_decode_rows.txt)."""
    rt = 1 if M <= 64 else -(-M // SKINNY_TILE_M)
    if target is None:
        target = _TARGET_WGS if rt == 1 else 2 * _TARGET_WGS
    blocks = N // _ROWS_PER_WG * rt
    s = 1
    while blocks * s < target and s < 16 and K % (_KCHUNK * s * 2) == 0:
        s *= 2
    return s


def skinny_ok(x: torch.Tensor, w: torch.Tensor, force: bool = False, max_m: int = SKINNY_MAX_M) -> bool:
    if not (SKINNY_ENABLED or force) or not x.is_cuda or x.dtype != torch.bfloat16:
        return False
    M, K = x.shape
    N = w.shape[0]
    return (0 < M <= max_m and N % _ROWS_PER_WG == 0 and K % _KCHUNK == 0 and x.stride(1) == 1
            and x.stride(0) % 8 == 0)


def norm_fusable(H: int) -> bool:
    """Hidden sizes the split-K + residual + RMSNorm kernel handles."""
    return H % 1024 == 0 and H <= 8192


def pack_weight(w: torch.Tensor) -> torch.Tensor:
    """Row-major ``[N, K]`` → block-packed layout for the decode GEMM (same size).

    For every 128-row n-block (one workgroup) and 128-deep k-step, the 32 KiB the workgroup
    consumes are contiguous: 8 row tiles x 4 k-blocks of 32, each a 1 KiB MFMA A-fragment in
    lane order (lane l = 16*g + r holds row r, k = 8g..8g+7).  A wave load instruction reads
    1 KiB and a workgroup sweeps a single linear stream (tools/gemm_lab.hip)."""
    N, K = w.shape
    assert N % 128 == 0 and K % 128 == 0
    # [nb, tile, r, ks, s, g, e] -> [nb, ks, tile, s, g, r, e]
    return w.view(N // 128, 8, 16, K // 128, 4, 4, 8).permute(0, 3, 1, 4, 5, 2, 6).contiguous().view(N, K)


def unpack_weight(wp: torch.Tensor) -> torch.Tensor:
    N, K = wp.shape
    return wp.view(N // 128, K // 128, 8, 4, 4, 16, 8).permute(0, 2, 5, 1, 3, 4, 6).contiguous().view(N, K)


# weights at least this large are streamed with non-temporal loads (gate_up, MoE w13, LM head)
NT_MIN_BYTES = 160 << 20
NT_BIT = 64


def _wmode(packed: Optional[torch.Tensor]) -> int:
    if packed is None:
        return 0
    return PACKED_BIT | (NT_BIT if packed.numel() * packed.element_size() >= NT_MIN_BYTES else 0)


def linear(x: torch.Tensor, w: torch.Tensor, out: Optional[torch.Tensor] = None,
           packed: Optional[torch.Tensor] = None, max_m: int = SKINNY_MAX_M) -> torch.Tensor:
    """bf16 out [M, N]; ``packed`` = :func:`pack_weight` (w) streamed instead of ``w`` when given;
    the skinny kernel up to ``max_m`` rows (decode callers: :data:`DECODE_MAX_M`)."""
    if not skinny_ok(x, w, max_m=max_m):
        if w.is_meta:  # packed-only weights (LlamaForCausalLM.pack_decode_weights): prefill on them
            from . import gemm_prefill
            return gemm_prefill.linear(x, w, out=out, packed=packed)
        # torch.mm into a preallocated output: hipBLASLt picks a faster kernel for the 8B QKV
        # prefill shape than through F.linear (288 vs 344 us at 8192 rows; the other
        # projections are equal: profiles/r2_prefill_gemm_lab.txt)
        if out is None:
            out = torch.empty((x.shape[0], w.shape[0]), dtype=x.dtype, device=x.device)
        return torch.mm(x, w.t(), out=out)
    M, K = x.shape
    N = w.shape[0]
    if out is None:
        out = torch.empty((M, N), dtype=x.dtype, device=x.device)
    src = packed if packed is not None else w
    # too few 128-row n-blocks for the chip (the 70B TP=8 LM-head shard: 126): 64-row n-blocks
    half = packed is not None and M <= SKINNY_MAX_M and N // _ROWS_PER_WG < _TARGET_WGS
    native.call("pk_skinny_gemm", out.data_ptr(), 0, x.data_ptr(), src.data_ptr(), M, N, K, x.stride(0),
                out.stride(0), 1, 0 | _wmode(packed) | (HALF_BIT if half else 0), native.stream_ptr())
    return out


# TP decode: each row-parallel projection runs as this many column-chunk GEMMs on the compute stream,
# each chunk's fused collective on the comm stream behind an event after ITS GEMM -- the collective
# of chunk c overlaps the GEMM of chunk c + 1 (1: one GEMM, then one collective)
# Measured: the chunked GEMMs + stream fork / join cost 16 us per 70B TP=8 layer on the GEMM side
# alone (per-rank step 7.38 vs 6.07 ms with 2 chunks, 10.1 ms with 4; profiles/r5_tp_overlap.md) --
# more than the xGMI time they could hide: one GEMM + one collective by default
TP_DECODE_CHUNKS = int(os.environ.get("POLYKEY_TP_DECODE_CHUNKS", "1"))


def partial_tiling(N: int, K: int, M: int, packed: Optional[torch.Tensor], half: bool):
    """(split, half) of a split-K slab projection: ``half`` (64-row n-blocks at half the split)
    holds only for packed weights below :data:`NT_MIN_BYTES`.  Shared by :func:`linear_partial`
    and :func:`push_projection`, whose slabs must be bit-identical."""
    half = half and packed is not None and packed.numel() * packed.element_size() < NT_MIN_BYTES
    S = choose_split(N, K, M)
    return (max(1, S // 2) if half else S), half


def linear_partial(x: torch.Tensor, w: torch.Tensor, ws: torch.Tensor, S: Optional[int] = None,
                   packed: Optional[torch.Tensor] = None, half: bool = False) -> Partial:
    """Split-K fp32 slabs into workspace ``ws`` (fp32, >= S*M*N).  ``half`` (packed W): 64-row
    n-blocks at half the default split -- the same grid, half the slab bytes."""
    M, K = x.shape
    N = w.shape[0]
    S_auto, half = partial_tiling(N, K, M, packed, half)
    S = S_auto if S is None else S
    assert ws.numel() >= S * M * N, "split-K workspace too small"
    src = packed if packed is not None else w
    native.call("pk_skinny_gemm", 0, ws.data_ptr(), x.data_ptr(), src.data_ptr(), M, N, K, x.stride(0), N, S,
                1 | _wmode(packed) | (HALF_BIT if half else 0), native.stream_ptr())
    return Partial(ws, S, M, N)


def linear_silu(x: torch.Tensor, w_gu_interleaved: torch.Tensor, ws: Optional[torch.Tensor] = None,
                packed: Optional[torch.Tensor] = None, norm: Optional[NormIn] = None,
                rowscale: Optional[RowScale] = None, max_m: int = SKINNY_MAX_M) -> torch.Tensor:
    """silu(x @ Wg^T) * (x @ Wu^T) with interleaved gate/up rows → [M, I].  With ``norm``,
    ``x`` is the residual stream and the RMSNorm is applied in the kernel's prologue (S = 1);
    with ``rowscale`` the norm is folded (W pre-multiplied, rows scaled in the epilogue)."""
    if norm is not None or rowscale is not None:
        M, K = x.shape
        N = w_gu_interleaved.shape[0]
        out = torch.empty((M, N // 2), dtype=x.dtype, device=x.device)
        Sg = gate_up_split(N, K, M) if rowscale is not None and M <= FUSED_MAX_M else 1
        if Sg > 1 and ws is not None and ws.numel() >= Sg * M * N:
            # split over K when its n-blocks cannot fill the chip (the 70B TP=8 shard), then one
            # SiLU reduce launch over the slabs
            p = linear_partial_rowscale(x, w_gu_interleaved, ws, rowscale, S=Sg, packed=packed)
            native.call("pk_splitk_reduce", out.data_ptr(), p.buf.data_ptr(), Sg, M, N, out.stride(0), 1,
                        native.stream_ptr())
            return out
        _launch_ex(MODE_SILU, x, w_gu_interleaved, packed, 1, out=out, norm=norm, rowscale=rowscale)
        return out
    if not skinny_ok(x, w_gu_interleaved, max_m=max_m):
        if w_gu_interleaved.is_meta:  # packed-only weights: fused SiLU in the prefill GEMM epilogue
            from . import gemm_prefill
            return gemm_prefill.linear(x, w_gu_interleaved, packed=packed, silu=True)
        return silu_and_mul_interleaved(linear(x, w_gu_interleaved))
    M, K = x.shape
    N = w_gu_interleaved.shape[0]
    out = torch.empty((M, N // 2), dtype=x.dtype, device=x.device)
    S = choose_split(N, K, M)
    if S == 1 or ws is None or ws.numel() < S * M * N:
        src = packed if packed is not None else w_gu_interleaved
        native.call("pk_skinny_gemm", out.data_ptr(), 0, x.data_ptr(), src.data_ptr(), M, N, K,
                    x.stride(0), out.stride(0), 1, 2 | _wmode(packed), native.stream_ptr())
    else:
        p = linear_partial(x, w_gu_interleaved, ws, S, packed=packed)
        native.call("pk_splitk_reduce", out.data_ptr(), ws.data_ptr(), S, M, N, out.stride(0), 1, native.stream_ptr())
    return out


def linear_partial_rowscale(x: torch.Tensor, w: torch.Tensor, ws: torch.Tensor, rowscale: RowScale,
                            S: Optional[int] = None, packed: Optional[torch.Tensor] = None,
                            half: bool = False) -> Partial:
    """:func:`linear_partial` of a folded-norm projection: slabs of rinv[m] * (x @ W'^T).
    ``half`` (packed W): 64-row n-blocks at half the default split."""
    M, K = x.shape
    N = w.shape[0]
    S, half = _rowscale_tiling(N, K, M, packed, half, S)
    assert ws.numel() >= S * M * N, "split-K workspace too small"
    _launch_ex(MODE_PARTIAL | (HALF_BIT if half else 0), x, w, packed, S, ws=ws, rowscale=rowscale)
    return Partial(ws, S, M, N)


def _rowscale_tiling(N: int, K: int, M: int, packed: Optional[torch.Tensor], half: bool, S: Optional[int]):
    """(split, half) of :func:`linear_partial_rowscale` (shared with its collective-carrying form)."""
    half = half and packed is not None and packed.numel() * packed.element_size() < NT_MIN_BYTES
    if S is None:
        S = choose_split(N, K, M)
        if half:
            S = max(1, S // 2)
    return S, half


# the carried launch with each workgroup running a collective item and then a consumer tile (A/B)
CAR_PAIRED = True  # (separate workgroups measured slower: profiles/r6_carry.md)


def linear_partial_rowscale_car(car_dev, pending: Partial, residual: torch.Tensor, parts: torch.Tensor,
                                w: torch.Tensor, ws: torch.Tensor, eps: float, flow: torch.Tensor,
                                packed: torch.Tensor, S: Optional[int] = None, half: bool = False):
    """ONE launch (csrc/kernels/car_gemm.hip): the two-shot TP collective of ``pending`` (the
    row-parallel projection's split-K slabs) into ``residual`` / ``parts`` -- exactly
    ``custom_ar.reduce_residual`` -- and the folded-norm projection that consumes that residual --
    exactly :func:`linear_partial_rowscale` (same tiling and split, bit-identical slabs) -- whose
    tiles stream their weights while the collective runs and wait only for the chunk groups they
    read.  ``car_dev``: ``CustomAllReduce.device_ctx()``; ``flow``: int32 >= :data:`FLOW_WORDS`,
    zeroed once, left zeroed.  Returns (the parts view [N / 256, M], the consumer's slabs)."""
    M, N = residual.shape
    Nc, K = w.shape
    assert K == N and pending.M == M and pending.N == N and residual.is_contiguous()
    S, half = _rowscale_tiling(Nc, K, M, packed, half, S)
    assert ws.numel() >= S * M * Nc and flow.numel() >= FLOW_WORDS and flow.dtype == torch.int32
    # (ws may be pending's own buffer: a consumer tile stores its slabs only after the whole
    # collective -- every slab read included -- has taken its tickets)
    g = GemmArgs()
    g.partial, g.A, g.W = ws.data_ptr(), residual.data_ptr(), packed.data_ptr()
    g.M, g.N, g.K, g.lda, g.ldo, g.S = M, Nc, K, N, Nc, S
    g.row_scale, g.nrm_parts, g.nrm_nparts, g.eps = 1, parts.data_ptr(), N // 256, float(eps)
    native.call("pk_car_gemm", ctypes.cast(car_dev, ctypes.c_void_p), pending.buf.data_ptr(), pending.S,
                residual.data_ptr(), parts.data_ptr(), M, N, ctypes.byref(g), 1 if half else 2, int(CAR_PAIRED),
                flow.data_ptr(), native.stream_ptr())
    return parts.view(-1)[: (N // 256) * M].view(N // 256, M), Partial(ws, S, M, Nc)


_CUS: dict = {}


def device_cus(dev: torch.device) -> int:
    """Compute units of ``dev`` (256 on an MI355X), queried once per device."""
    i = dev.index if dev.index is not None else torch.cuda.current_device()
    if i not in _CUS:
        _CUS[i] = torch.cuda.get_device_properties(i).multi_processor_count
    return _CUS[i]


# fused-launch hand-off buffer (csrc/kernels/gemm_skinny.hip kFlowWords): 64 tickets + 64 consumer
# counts (256 B apart), the error word, then the split gate_up's per-n-block counters
FLOW_WORDS = 128 * 64 + 64 + 1024


_FUSED_ERR: Optional[int] = None


def fused_err_word() -> int:
    """Address of the fused launches' sticky timeout word (host-mapped pinned memory, allocated
    once per process; every later fused launch reports into it)."""
    global _FUSED_ERR
    if _FUSED_ERR is None:
        fn = native.lib().pk_fused_err_word
        fn.restype, fn.argtypes = ctypes.c_void_p, []
        _FUSED_ERR = fn()
        if not _FUSED_ERR:
            raise native.KernelError("pk_fused_err_word: hipHostMalloc failed")
    return _FUSED_ERR


class FusedHandoffError(RuntimeError):
    """An in-launch hand-off of a fused decode launch timed out: its outputs are invalid."""


def check_fused() -> None:
    """Raise :class:`FusedHandoffError` once any in-launch hand-off wait of a fused decode launch
    timed out: that launch's outputs were computed from data that had not arrived (cannot happen
    while every workgroup of the grid is resident; another process on the same GPU could break
    that).  A plain read of host memory, no GPU sync: the engine calls it every step like the
    collectives' error words, and falls back to the two-launch path (LLMEngine)."""
    if _FUSED_ERR is not None and ctypes.c_int.from_address(_FUSED_ERR).value != 0:
        raise FusedHandoffError("a fused decode launch's in-kernel hand-off timed out (results invalid)")


def clear_fused_error() -> None:
    """Re-arm the sticky word (after the caller has stopped using the fused launches)."""
    if _FUSED_ERR is not None:
        fn = native.lib().pk_clear_fused_err
        fn.restype, fn.argtypes = None, []
        fn()


def disable_fused() -> None:
    """Every later decode step takes the two-launch path (QKV | attention, gate_up | down)."""
    global MLP_FUSED, QKV_ATTN_FUSED
    MLP_FUSED = False
    QKV_ATTN_FUSED = False


def set_fused_spin_limit(n: int) -> None:
    """Tests: polls a fused consumer makes before declaring its hand-off lost (0: default; < 0:
    every wait reports a lost hand-off, to drive the engine's fallback deterministically)."""
    fn = native.lib().pk_set_fused_spin_limit
    fn.restype, fn.argtypes = None, [ctypes.c_int]
    fn(int(n))


def down_kr(N: int, K: int, M: int) -> int:
    """n-block height of a decode down projection's tiles (in 64 rows; csrc gemm_skinny.hip
    down_kr): 1 when 128-row tiles at its split would be fewer than 192 workgroups (8B: 32 x 4,
    70B TP=8: 64 x 2 -> 256 tiles of 64 rows), else 2.  The fused MLP and the two-launch chain
    use the same, so their slabs are bit-identical."""
    return 1 if (N // _ROWS_PER_WG) * choose_split(N, K, M) < _TARGET_WGS else 2


def linear_down(h: torch.Tensor, w: torch.Tensor, ws: torch.Tensor, packed: Optional[torch.Tensor]) -> Partial:
    """The decode down projection as the fused MLP launch tiles it (split :func:`choose_split`,
    n-blocks of :func:`down_kr` x 64 rows) -> fp32 slabs."""
    M, K = h.shape
    N = w.shape[0]
    S = choose_split(N, K, M)
    if packed is not None and down_kr(N, K, M) == 1 and M <= FUSED_MAX_M:
        assert ws.numel() >= S * M * N, "split-K workspace too small"
        native.call("pk_skinny_gemm", 0, ws.data_ptr(), h.data_ptr(), packed.data_ptr(), M, N, K, h.stride(0), N, S,
                    1 | PACKED_BIT | HALF_BIT, native.stream_ptr())
        return Partial(ws, S, M, N)
    return linear_partial(h, w, ws, S, packed=packed)


class PushTarget(NamedTuple):
    """Where a MODE_PUSH epilogue stores (custom_ar.CustomAllReduce.push_target): the device array
    of every TP rank's IPC buffer, this rank, the group size, the bytes of one data slot."""
    peers: int
    rank: int
    world: int
    slot_bytes: int


def push_projection(x: torch.Tensor, w: torch.Tensor, ws: torch.Tensor, packed: torch.Tensor,
                    counters: torch.Tensor, target: PushTarget, down: bool = False,
                    split: Optional[int] = None) -> int:
    """A row-parallel TP decode projection x @ w^T whose epilogue drives its collective: tiled and
    split exactly as :func:`linear_down` (``down``) or :func:`linear_partial` ``half=True`` (the o
    projection), so its slabs are bit-identical; the last split of every n-block stores bf16(sum of
    the slabs) into the owner rank's input slot and stamps the owner's push flag.  ``counters``:
    int32 >= N / 64, zeroed once (left zeroed).  Returns the n-block width the owners' collective
    needs (custom_ar.reduce_residual_pushed)."""
    M, K = x.shape
    N = w.shape[0]
    if down:
        S = choose_split(N, K, M)
        half = down_kr(N, K, M) == 1 and M <= FUSED_MAX_M
    else:
        # the unpushed chain's o projection is linear_partial(half=True): the same helper picks
        # both tilings, so they cannot drift apart
        S, half = partial_tiling(N, K, M, packed, True)
    S = split or S  # (tools/push_probe.py: other splits, not bit-identical to the serving chain)
    nbc = 64 if half else 128
    assert ws.numel() >= S * M * N and counters.numel() >= N // 64 and counters.dtype == torch.int32
    _launch_ex(MODE_PUSH | (HALF_BIT if half else 0), x, w, packed, S, ws=ws, counters=counters,
               push_peers=target.peers, push_bytes=target.slot_bytes, push_rank=target.rank,
               push_world=target.world)
    return nbc


def gate_up_split(N2: int, K: int, M: int) -> int:
    """K split of a decode gate_up projection (1: the single-pass SiLU epilogue).  Its n-blocks
    alone fill the chip for 8B (224) but not for the 70B TP=8 shard (56: split 4)."""
    return choose_split(N2, K, M)


def fused_rows_ok(M: int, nparts: int) -> bool:
    """Row counts the fused decode launches take: one tile of up to 64 rows, or of 128 rows when
    the row scale has at most :data:`FUSED_MT8_MAX_PARTS` norm parts."""
    return 0 < M <= SKINNY_MAX_M or (M <= FUSED_MAX_M and nparts <= FUSED_MT8_MAX_PARTS)


def mlp_fused_ok(x: torch.Tensor, gate_up_packed: Optional[torch.Tensor], down_packed: Optional[torch.Tensor],
                 nparts: int = 0) -> bool:
    """Shapes the fused decode MLP launch (:func:`mlp_fused`) takes (``nparts``: norm parts of
    its row scale)."""
    if gate_up_packed is None or down_packed is None or not x.is_cuda or not MLP_FUSED:
        return False
    M, K = x.shape
    if not fused_rows_ok(M, nparts):
        return False
    N2, I = gate_up_packed.shape[0], down_packed.shape[1]
    S = choose_split(down_packed.shape[0], I, M)
    if gate_up_split(N2, K, M) > 1:
        return False
    # one workgroup per CU, each a gate_up tile then a down tile: above 256 tiles (70B on one GPU:
    # 448 gate_up tiles) the fused launch measured 8 % slower end to end (profiles/r2_decode_ab.txt)
    return (N2 == 2 * I and N2 % 128 == 0 and K % _KCHUNK == 0
            and down_packed.shape[0] % 128 == 0 and I % (_KCHUNK * S) == 0 and (I // S) % 64 == 0 and S <= 64
            and gate_up_packed.shape[1] == K and N2 // 128 <= device_cus(x.device)
            and (down_packed.shape[0] // (64 * down_kr(down_packed.shape[0], I, M))) * S <= device_cus(x.device))


def mlp_fused(x: torch.Tensor, gate_up_packed: torch.Tensor, down_packed: torch.Tensor, rowscale: RowScale,
              ws: torch.Tensor, flow: torch.Tensor) -> Partial:
    """Decode MLP in ONE launch (csrc/kernels/gemm_skinny.hip mlp_fused_kernel):
    h = silu/mul of rinv * (x @ Wgu'^T) (folded norm, interleaved packed gate/up), then the down
    projection's fp32 split-K slabs of h @ Wd^T in ``ws``.  Down workgroups stream their first
    weight k-steps while gate_up finishes and wait on per-K-slice tickets in ``flow`` (int32,
    >= :data:`FLOW_WORDS`, zeroed once; every launch leaves it zeroed).  Returns the down slabs."""
    M, K = x.shape
    N2, I = gate_up_packed.shape[0], down_packed.shape[1]
    N = down_packed.shape[0]
    S = choose_split(N, I, M)
    assert ws.numel() >= S * M * N and flow.numel() >= FLOW_WORDS and flow.dtype == torch.int32
    assert gate_up_split(N2, K, M) == 1, "the fused MLP takes unsplit gate_up shapes (mlp_fused_ok)"
    h = torch.empty((M, I), dtype=x.dtype, device=x.device)
    gu = GemmArgs()
    gu.out, gu.A, gu.W = h.data_ptr(), x.data_ptr(), gate_up_packed.data_ptr()
    gu.M, gu.N, gu.K, gu.lda, gu.ldo, gu.S = M, N2, K, x.stride(0), h.stride(0), 1
    gu.row_scale, gu.nrm_parts, gu.nrm_nparts, gu.eps = 1, rowscale.parts.data_ptr(), rowscale.parts.shape[0], \
        float(rowscale.eps)
    dn = GemmArgs()
    dn.partial, dn.A, dn.W = ws.data_ptr(), h.data_ptr(), down_packed.data_ptr()
    dn.M, dn.N, dn.K, dn.lda, dn.ldo, dn.S = M, N, I, h.stride(0), N, S
    native.call("pk_mlp_fused", ctypes.byref(gu), ctypes.byref(dn), flow.data_ptr(), native.stream_ptr())
    return Partial(ws, S, M, N)


QKV_ATTN_FUSED = os.environ.get("POLYKEY_QKV_ATTN_FUSED", "1") == "1"


def qkv_attn_fused(x: torch.Tensor, qkv_packed: torch.Tensor, rowscale: RowScale, ws: torch.Tensor,
                   positions: torch.Tensor, cos_sin: torch.Tensor, k_cache: torch.Tensor, v_cache: torch.Tensor, md,
                   scale: float, nq: int, nkv: int, flow: torch.Tensor, S: Optional[int] = None) -> torch.Tensor:
    """Decode layer front half in ONE launch (csrc/kernels/decode_fused.hip): the folded-norm
    QKV projection's split-K slabs (``ws``), handed in-launch to the decode attention that
    reduces them, applies RoPE, writes the new k / v to the paged cache and attends.  Same
    result as :func:`linear_partial_rowscale` + ``attention.paged_decode_from_qkv``.  ``flow``:
    int32 >= :data:`FLOW_WORDS`, zeroed once, left zeroed.  Returns [M, nq * 128] bf16."""
    M, K = x.shape
    N = qkv_packed.shape[0]
    S = S or choose_split(N, K, M)
    assert ws.numel() >= S * M * N and flow.numel() >= FLOW_WORDS and flow.dtype == torch.int32
    assert md.num_prefill == 0 and md.num_decode == M and k_cache.shape[-1] == 128
    from . import attention as _attn
    _attn.apply_decode_fill()
    out = torch.empty((M, nq * 128), dtype=torch.bfloat16, device=x.device)
    a = GemmArgs()
    a.partial, a.A, a.W = ws.data_ptr(), x.data_ptr(), qkv_packed.data_ptr()
    a.M, a.N, a.K, a.lda, a.ldo, a.S = M, N, K, x.stride(0), N, S
    a.row_scale, a.nrm_parts, a.nrm_nparts, a.eps = 1, rowscale.parts.data_ptr(), rowscale.parts.shape[0], \
        float(rowscale.eps)
    bt = md.decode_block_tables
    native.call("pk_qkv_attn_fused", ctypes.byref(a), out.data_ptr(), positions.data_ptr(), cos_sin.data_ptr(),
                md.slot_mapping.data_ptr(), k_cache.data_ptr(), v_cache.data_ptr(), bt.data_ptr(),
                md.decode_context_lens.data_ptr(), native.ptr(md.decode_part_o) or 0,
                native.ptr(md.decode_part_ml) or 0, nq, nkv, k_cache.shape[2], bt.stride(0), out.stride(0),
                float(scale), int(md.decode_max_ctx), flow.data_ptr(), native.stream_ptr())
    return out


def fold_norm(w: torch.Tensor, norm_weight: torch.Tensor) -> torch.Tensor:
    """W' = W diag(norm_weight): the RMSNorm weight of the projection's input folded into its
    columns (bf16), for the row-scaled decode GEMM (:class:`RowScale`)."""
    return (w.float() * norm_weight.float()[None, :]).to(w.dtype)


PART_COLS = 512  # columns per sum-of-squares part written by residual_parts


def residual_parts(p: Optional[Partial], residual: torch.Tensor, parts: torch.Tensor) -> torch.Tensor:
    """residual += sum of ``p``'s slabs (bf16, in place; ``p`` None: unchanged) and
    parts [H/512, M] = per-512-column sums of squares of the new residual rows."""
    M, H = residual.shape
    n = H // PART_COLS
    assert parts.numel() >= n * M and residual.is_contiguous()
    if not residual.is_cuda:
        if p is not None:
            residual.copy_((residual.float() + p.view().sum(0).to(torch.bfloat16).float()).to(residual.dtype))
        parts.view(-1)[: n * M].copy_(residual.float().view(M, n, PART_COLS).pow(2).sum(-1).t().reshape(-1))
        return parts.view(-1)[: n * M].view(n, M)
    native.call("pk_residual_parts", residual.data_ptr(), 0 if p is None else p.buf.data_ptr(), 0 if p is None else p.S,
                M, H, parts.data_ptr(), native.stream_ptr())
    return parts.view(-1)[: n * M].view(n, M)


def silu_reduce(p: Partial, out: torch.Tensor) -> torch.Tensor:
    """h = SiLU(gate) * up of the summed slabs of an interleaved gate/up projection (the split
    gate_up's reduce launch, as :func:`linear_silu` runs it) into ``out`` [M, N / 2]."""
    native.call("pk_splitk_reduce", out.data_ptr(), p.buf.data_ptr(), p.S, p.M, p.N, out.stride(0), 1,
                native.stream_ptr())
    return out


def reduce_partial(p: Partial, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    if out is None:
        out = torch.empty((p.M, p.N), dtype=torch.bfloat16, device=p.buf.device)
    native.call("pk_splitk_reduce", out.data_ptr(), p.buf.data_ptr(), p.S, p.M, p.N, out.stride(0), 0,
                native.stream_ptr())
    return out


def partial_add_rms_norm(p: Partial, residual: torch.Tensor, weight: torch.Tensor, eps: float,
                         out: Optional[torch.Tensor] = None):
    """residual += sum(p) (bf16), x = rms_norm(residual) * w.  Returns (x, residual)."""
    if out is None:
        out = torch.empty_like(residual)
    native.call("pk_splitk_add_rmsnorm", out.data_ptr(), residual.data_ptr(), p.buf.data_ptr(), weight.data_ptr(),
                p.S, p.M, p.N, float(eps), native.stream_ptr())
    return out, residual


def partial_add_rms_norm_route(p: Partial, residual: torch.Tensor, weight: torch.Tensor, eps: float,
                               router: torch.Tensor, k: int, renorm: bool = True):
    """:func:`partial_add_rms_norm` that also routes every normalised row (MoE): router logits
    (bf16), softmax, top-k → (x, residual, ids [M, k] int32, weights [M, k] fp32)."""
    M, H = residual.shape
    E = router.shape[0]
    out = torch.empty_like(residual)
    ids = torch.empty((M, k), dtype=torch.int32, device=residual.device)
    w = torch.empty((M, k), dtype=torch.float32, device=residual.device)
    native.call("pk_splitk_add_rmsnorm_route", out.data_ptr(), residual.data_ptr(), p.buf.data_ptr(),
                weight.data_ptr(), p.S, p.M, p.N, float(eps), router.data_ptr(), E, k, int(renorm), ids.data_ptr(),
                w.data_ptr(), native.stream_ptr())
    return out, residual, ids, w


def silu_and_mul_interleaved(x: torch.Tensor, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """silu(gate) * up of gate/up columns interleaved by 16 → [..., I]; ``out``: a contiguous
    destination (e.g. a row slice of a larger buffer) written in place."""
    if not x.is_cuda:
        y = reference.silu_and_mul_interleaved(x)
        return y if out is None else out.copy_(y)
    I2 = x.shape[-1]
    T = x.numel() // I2
    if out is None:
        out = torch.empty(x.shape[:-1] + (I2 // 2,), dtype=x.dtype, device=x.device)
    assert out.is_contiguous() and out.numel() == T * (I2 // 2)
    native.call("pk_silu_and_mul_il", out.data_ptr(), x.data_ptr(), T, I2 // 2, native.stream_ptr())
    return out


def qkv_reduce_rope_cache(p: Partial, positions: torch.Tensor, cos_sin: torch.Tensor, k_cache: torch.Tensor,
                          v_cache: torch.Tensor, slots: torch.Tensor, nq: int, nkv: int) -> torch.Tensor:
    """Split-K QKV epilogue: sum slabs, RoPE q/k, write k/v to the paged cache → q [M, nq, 128]."""
    q = torch.empty((p.M, nq, 128), dtype=torch.bfloat16, device=p.buf.device)
    native.call("pk_qkv_reduce_rope_cache", q.data_ptr(), p.buf.data_ptr(), p.S, p.M, nq, nkv, positions.data_ptr(),
                cos_sin.data_ptr(), k_cache.data_ptr(), v_cache.data_ptr(), slots.data_ptr(), k_cache.shape[2],
                native.stream_ptr())
    return q
