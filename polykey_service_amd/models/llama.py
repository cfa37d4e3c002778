"""Llama-3 family decoder (8B / 70B; also the attention half of Mixtral), TP-aware.

Prefill (and decode batches above the fused kernels' limits), per layer on one rank (TP degree
``tp``; shapes for 8B TP1 / 70B TP8 in SURVEY.md §2.3):

    x, res = fused_add_rmsnorm(x, res)                       HIP  (csrc/kernels/norm_act.hip)
    qkv    = x @ Wqkv^T          column-parallel by heads     hipBLASLt, or the hand-written MFMA GEMM
                                                              on block-packed weights (gemm_prefill.hip)
    rope_and_cache(qkv)          rotate q,k in place, write the paged K / V cache (fragment-native
                                 32-token tiles, common.h kcache_off / vcache_off)   HIP
    a      = paged_attention(q)  varlen causal prefill over the cached prefix (MFMA) HIP
    o      = a @ Wo^T            row-parallel -> all-reduce (RCCL over xGMI; chunk-overlapped, or
                                 reduce-scatter / all-gather around the norms: sequence parallel)
    x, res = fused_add_rmsnorm(o, res)                       HIP
    h      = silu_and_mul(x @ Wgu^T)                         hipBLASLt / MFMA GEMM + HIP
    x      = h @ Wdown^T         row-parallel -> all-reduce

Decode (M <= 64 rows; ``_forward_rowscale``): the RMSNorm weights are folded into the block-packed
QKV / gate_up weights and every projection is the hand-written weight-streaming GEMM
(gemm_skinny.hip / skinny_tile.h), per layer

    qkv_attn_fused   QKV split-K slabs handed in-launch to the decode attention (RoPE, KV write)
    o-proj slabs  -> residual update + norm parts (TP: the fused xGMI collective, custom_ar)
    mlp_fused        gate_up + SiLU handed in-launch to the down projection's slabs
                  -> residual update + norm parts (TP: the fused collective)

Vocab-parallel embedding and LM head for TP>1 (logits all-gathered for sampling).
"""
from __future__ import annotations

import math
import os
from typing import List, Optional, Tuple

import torch
import torch.nn.functional as F
from torch import nn

from .. import ops
from ..ops import attention as attn_ops
from ..ops import gemm
from ..ops import gemm_prefill
from ..ops import moe as moe_ops
from ..ops import reference
from ..parallel import comm
from ..parallel.state import ParallelState, get_state
from ..utils import test_hooks
from .config import ModelConfig
from .weights import SafetensorsIndex, random_full, random_shard, shard_cols, shard_rows


# Decode (dense, block-packed weights): every RMSNorm weight is folded into the columns of the
# projection that consumes it and that projection scales its output rows by rinv, so the per-layer
# norm kernels shrink to residual updates (TP = 1) or to the fused TP collective (TP > 1).  Tests
# switch it off to compare against the normalised chain.
FOLD_NORM = True
# TP > 1 steps with at least SP_MIN_TOKENS tokens (prefill) run with a token-sharded residual
# stream: reduce-scatter / all-gather around the norms instead of all-reduces (_forward_sp).
SEQUENCE_PARALLEL = os.environ.get("POLYKEY_SEQUENCE_PARALLEL", "1") == "1"
SP_MIN_TOKENS = int(os.environ.get("POLYKEY_SP_MIN_TOKENS", "256"))


def _p(t: torch.Tensor) -> nn.Parameter:
    return nn.Parameter(t, requires_grad=False)


def _proj(x: torch.Tensor, w: torch.Tensor, ws: Optional[torch.Tensor],
          wp: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Column-parallel projection → bf16 (skinny split-K + reduce for decode-sized M).
    ``wp``: the block-packed copy of ``w`` streamed by the decode GEMM (None: row-major)."""
    if ws is not None and gemm.skinny_ok(x, w):
        S = gemm.choose_split(w.shape[0], x.shape[1], x.shape[0])
        if S > 1 and ws.numel() >= S * x.shape[0] * w.shape[0]:
            return gemm.reduce_partial(gemm.linear_partial(x, w, ws, S, packed=wp))
    return gemm.linear(x, w, packed=wp)


def _proj_out(x: torch.Tensor, w: torch.Tensor, ws: Optional[torch.Tensor], wp: Optional[torch.Tensor] = None,
              half: bool = False):
    """Row-parallel projection feeding a residual add + RMSNorm.  TP=1 decode returns the
    split-K partial slabs unreduced (the norm kernel sums them); TP>1 all-reduces bf16.
    ``half``: slabs from 64-row n-blocks at half the split (the o-projection: -0.7..1.5 % decode
    step, profiles/r2_decode_ab.txt)."""
    if get_state().tp_size == 1 and ws is not None and gemm.skinny_ok(x, w) and gemm.norm_fusable(w.shape[0]):
        S = gemm.choose_split(w.shape[0], x.shape[1], x.shape[0])
        if ws.numel() >= S * x.shape[0] * w.shape[0]:
            if half:
                return gemm.linear_partial(x, w, ws, packed=wp, half=True)
            return gemm.linear_partial(x, w, ws, S, packed=wp)
    if x.shape[0] > gemm.SKINNY_MAX_M:
        # prefill: the all-reduce of one row chunk overlaps the GEMM of the next
        return comm.tp_row_parallel_overlapped(x, w.shape[0],
                                               lambda rows, out: gemm.linear(rows, w, out=out, packed=wp),
                                               chunks=comm.overlap_chunks(x.shape[0]))
    return comm.tp_all_reduce(_proj(x, w, ws, wp))


LM_HEAD_SKINNY_MAX_M = 128
# above this many decode rows gate_up runs on hipBLASLt (+ the norm / SiLU kernels): 256 clients
# 19,030-19,728 -> 20,177-20,218 tok/s with 192 instead of 384 (profiles/r4_gate_up_rows_ab.jsonl)
GATE_UP_SKINNY_MAX_M = 192
# wide decode on the hand-written MFMA GEMM of prefill (gemm_prefill.hip, 256 x 256 tiles) reading
# the block-packed weights decode already holds, once its tiles -- counted by the rows they hold,
# a half-full row tile as half -- can fill the chip.  Llama-3-8B, tools/wide_gemm_probe.py (cold
# weights, profiles/r6_wide_gemm_probe.jsonl): gate_up + SiLU 105 vs hipBLASLt 123 us at 512 rows,
# the LM head 248 vs 306 us at 256 rows; whole decode step (tools/tp_solo.py --wide-min-tiles,
# r6_wide256/384.jsonl): gate_up on it at 448 / 512 rows 13.02 vs 13.42 / 13.82 vs 14.31 ms, but
# slower at 384 (12.34 vs 12.24: 168 row-weighted tiles), 256 (9.22 vs 9.00) and 200 rows
WIDE_MFMA_MIN_TILES = 180


def _wide_mfma_ok(x: torch.Tensor, packed: Optional[torch.Tensor]) -> bool:
    """Decode rows ``x`` times the block-packed ``packed`` on the prefill MFMA GEMM: a shape it
    tiles, with at least WIDE_MFMA_MIN_TILES row-weighted 256 x 256 tiles."""
    if packed is None or x.stride(1) != 1:
        return False
    N, K = packed.shape
    tiles = (N // gemm_prefill.BN) * x.shape[0] / gemm_prefill.BM
    return gemm_prefill.supported(N, K) and K % 128 == 0 and tiles >= WIDE_MFMA_MIN_TILES


def pack_folded(owner, name: str, norm_w: torch.Tensor, packed_only: bool) -> torch.Tensor:
    """Block-packed copy of ``owner.<name>`` with ``norm_w`` folded into its columns; with
    ``packed_only`` the row-major weight becomes a meta placeholder (freed before the next)."""
    src = getattr(owner, name)
    out = gemm.pack_weight(gemm.fold_norm(src, norm_w))
    if packed_only:
        setattr(owner, name, _p(torch.empty(src.shape, dtype=src.dtype, device="meta")))
    return out


def add_norm(pending, residual: torch.Tensor, w: torch.Tensor, eps: float):
    """residual += pending; x = rms_norm(residual) * w → (x, residual)."""
    if isinstance(pending, gemm.Partial):
        return gemm.partial_add_rms_norm(pending, residual, w, eps)
    if isinstance(pending, moe_ops.PendingCombine):
        return moe_ops.combine_add_rms_norm(pending, residual, w, eps)
    return ops.fused_add_rms_norm(pending, residual, w, eps)


class LlamaAttention(nn.Module):
    def __init__(self, cfg: ModelConfig, st: ParallelState):
        super().__init__()
        self.hd = cfg.head_dim
        self.nq = cfg.num_heads // st.tp_size
        self.nkv = cfg.num_kv_heads // st.tp_size
        assert self.nkv >= 1, "tp larger than the number of KV heads is not supported"
        self.scale = 1.0 / math.sqrt(self.hd)
        self.qkv = None
        self.o = None
        self.qkv_p = None  # block-packed decode copies (LlamaForCausalLM.pack_decode_weights)
        self.o_p = None
        self.qkv_pf = None  # block-packed with ln1 folded in (FOLD_NORM)
        # fault injection for the TP correctness tests (LlamaForCausalLM, POLYKEY_FAULT_DROP_PARTIAL):
        # this rank's o-projection input is zeroed, i.e. its partial never reaches the collective
        self.fault_drop = False

    def drop(self, a: torch.Tensor) -> torch.Tensor:
        return a.zero_() if self.fault_drop else a

    def forward(self, x: torch.Tensor, positions: torch.Tensor, md: attn_ops.AttnMetadata, cos_sin: torch.Tensor,
                kv: Tuple[torch.Tensor, torch.Tensor], ws: Optional[torch.Tensor] = None):
        """Returns the o-projection output: a bf16 tensor, or (decode, TP=1) an unreduced
        split-K :class:`~polykey_service_amd.ops.gemm.Partial` consumed by the next norm."""
        T = x.shape[0]
        k_cache, v_cache = kv
        S = gemm.choose_split(self.qkv.shape[0], x.shape[1], T)
        if ws is not None and gemm.skinny_ok(x, self.qkv) and S > 1 and ws.numel() >= S * T * self.qkv.shape[0]:
            p = gemm.linear_partial(x, self.qkv, ws, S, packed=self.qkv_p)
            if md.num_prefill == 0:
                # pure decode: the attention kernel itself reduces the QKV slabs, applies RoPE
                # and writes the new k / v into the paged cache
                a = attn_ops.paged_decode_from_qkv(p, positions, cos_sin, k_cache, v_cache, md, self.scale,
                                                   self.nq, self.nkv)
                return _proj_out(self.drop(a), self.o, ws, self.o_p, half=True)
            # split-K QKV whose epilogue kernel also applies RoPE and writes the KV cache
            q = gemm.qkv_reduce_rope_cache(p, positions, cos_sin, k_cache, v_cache, md.slot_mapping, self.nq,
                                           self.nkv)
        else:
            return _proj_out(self.drop(self.attend(gemm.linear(x, self.qkv, packed=self.qkv_p), positions, md,
                                                   cos_sin, kv)), self.o, ws, self.o_p)
        a = attn_ops.paged_attention(q, k_cache, v_cache, md, self.scale)
        return _proj_out(self.drop(a), self.o, ws, self.o_p, half=True)

    def attend(self, qkv: torch.Tensor, positions: torch.Tensor, md: attn_ops.AttnMetadata, cos_sin: torch.Tensor,
               kv: Tuple[torch.Tensor, torch.Tensor]) -> torch.Tensor:
        """RoPE + KV-cache write + paged attention from a projected [T, (nq + 2 nkv) hd] qkv."""
        k_cache, v_cache = kv
        attn_ops.rope_and_cache(qkv, positions, cos_sin, k_cache, v_cache, md.slot_mapping, self.nq, self.nkv,
                                self.hd)
        q = qkv.view(qkv.shape[0], self.nq + 2 * self.nkv, self.hd)[:, :self.nq]
        return attn_ops.paged_attention(q, k_cache, v_cache, md, self.scale)


class LlamaMLP(nn.Module):
    def __init__(self):
        super().__init__()
        self.gate_up = None
        self.down = None
        self.gate_up_p = None
        self.down_p = None
        self.gate_up_pf = None  # block-packed with ln2 folded in (FOLD_NORM)

    def forward(self, x: torch.Tensor, ws: Optional[torch.Tensor] = None):
        h = gemm.linear_silu(x, self.gate_up, ws, packed=self.gate_up_p)  # gate/up rows interleaved by 16
        return _proj_out(h, self.down, ws, self.down_p)


class LlamaLayer(nn.Module):
    def __init__(self, cfg: ModelConfig, st: ParallelState, mlp: nn.Module):
        super().__init__()
        self.attn = LlamaAttention(cfg, st)
        self.mlp = mlp
        self.ln1 = None
        self.ln2 = None
        self.eps = cfg.rms_eps


class LlamaForCausalLM(nn.Module):
    """Dense Llama; :class:`~polykey_service_amd.models.mixtral.MixtralForCausalLM` swaps the MLP."""

    def __init__(self, cfg: ModelConfig, st: Optional[ParallelState] = None, dtype=torch.bfloat16,
                 device: Optional[torch.device] = None):
        super().__init__()
        self.cfg = cfg
        self.st = st or get_state()
        self.dtype = dtype
        self.device = device or self.st.device
        tp = self.st.tp_size
        assert cfg.num_heads % tp == 0 and cfg.num_kv_heads % tp == 0 and cfg.intermediate_size % tp == 0
        self.vocab_local = (cfg.vocab_size + tp - 1) // tp
        if tp > 1:
            # vocab shards padded to 128 rows: the LM-head shard stays on the block-packed decode
            # GEMM (128256 / 8 = 16032 rows -> 16128; Mixtral 32000 / 8 -> 4096); the zero rows
            # give logits past the vocabulary that compute_logits drops
            self.vocab_local = (self.vocab_local + 127) // 128 * 128
        self.vocab_start = self.st.tp_rank * self.vocab_local
        self.layers = nn.ModuleList([LlamaLayer(cfg, self.st, self._make_mlp(i)) for i in range(cfg.num_layers)])
        # POLYKEY_FAULT_DROP_PARTIAL=<layer>,<tp rank>: a deliberately wrong TP model (that rank's
        # attention partial of that layer is dropped) -- the TP=8 correctness test must fail on it.
        # Honoured only with POLYKEY_TEST_HOOKS=1, and logged at ERROR (utils/test_hooks.py)
        fault = test_hooks.get("POLYKEY_FAULT_DROP_PARTIAL")
        if fault:
            li, rk = (int(v) for v in fault.split(","))
            if rk == self.st.tp_rank and 0 <= li < cfg.num_layers:
                self.layers[li].attn.fault_drop = True
        self.embed = None
        self.norm = None
        self.lm_head = None
        self.lm_head_p = None  # block-packed decode copy (pack_decode_weights)
        self.register_buffer("cos_sin", reference.rope_cos_sin_cache(cfg.max_position, cfg.head_dim, cfg.rope_theta,
                                                                      cfg.rope_scaling, device=self.device),
                             persistent=False)

    def _make_mlp(self, layer: int) -> nn.Module:
        return LlamaMLP()

    # ------------------------------------------------------------------ weights
    def _vocab_pad(self, t: torch.Tensor) -> torch.Tensor:
        tp = self.st.tp_size
        pad = self.vocab_local * tp - t.shape[0]
        return torch.cat([t, t.new_zeros((pad,) + t.shape[1:])]) if pad else t

    def init_random(self, seed: int = 0) -> "LlamaForCausalLM":
        """Random weights, drawn shard-locally (``weights.random_shard``): every TP degree holds
        slices of the same logical tensors, and a rank draws only its own shard."""
        cfg, st, dev, dt = self.cfg, self.st, self.device, self.dtype
        H, hd, std = cfg.hidden_size, cfg.head_dim, cfg.init_std
        tp, r = st.tp_size, st.tp_rank
        self._seed = seed
        rows = lambda name, shape: random_shard(name, shape, std, seed, dev, dt, r, tp, 0)
        cols = lambda name, shape: random_shard(name, shape, std, seed, dev, dt, r, tp, 1)
        vocab = lambda name: random_shard(name, (cfg.vocab_size, H), std, seed, dev, dt, r, tp, 0,
                                          pad_to=self.vocab_local)
        self.embed = _p(vocab("embed").contiguous())
        self.norm = _p(torch.ones(H, dtype=dt, device=dev))
        self.lm_head = self.embed if cfg.tie_embeddings else _p(vocab("lm_head").contiguous())
        for i, layer in enumerate(self.layers):
            q = rows(f"l{i}.q", (cfg.num_heads * hd, H))
            k = rows(f"l{i}.k", (cfg.num_kv_heads * hd, H))
            v = rows(f"l{i}.v", (cfg.num_kv_heads * hd, H))
            layer.attn.qkv = _p(torch.cat([q, k, v]).contiguous())
            del q, k, v
            layer.attn.o = _p(cols(f"l{i}.o", (H, cfg.num_heads * hd)).contiguous())
            layer.ln1 = _p(torch.ones(H, dtype=dt, device=dev))
            layer.ln2 = _p(torch.ones(H, dtype=dt, device=dev))
            self._init_mlp_random(i, layer.mlp, rows, cols)
        return self

    def _init_mlp_random(self, i: int, mlp: nn.Module, rows, cols) -> None:
        cfg = self.cfg
        H, I = cfg.hidden_size, cfg.intermediate_size
        g = rows(f"l{i}.gate", (I, H))
        u = rows(f"l{i}.up", (I, H))
        mlp.gate_up = _p(gemm.interleave_gate_up(g, u).contiguous())
        del g, u
        mlp.down = _p(cols(f"l{i}.down", (H, I)).contiguous())

    def load_hf(self, path: str) -> "LlamaForCausalLM":
        idx = SafetensorsIndex(path)
        cfg, dev, dt = self.cfg, self.device, self.dtype
        tp, r = self.st.tp_size, self.st.tp_rank
        get = lambda n: idx.get(n).to(device=dev, dtype=dt)
        self.embed = _p(shard_rows(self._vocab_pad(get("model.embed_tokens.weight")), r, tp).contiguous())
        self.norm = _p(get("model.norm.weight"))
        if idx.has("lm_head.weight") and not cfg.tie_embeddings:
            self.lm_head = _p(shard_rows(self._vocab_pad(get("lm_head.weight")), r, tp).contiguous())
        else:
            self.lm_head = self.embed
        for i, layer in enumerate(self.layers):
            p = f"model.layers.{i}."
            q, k, v = (shard_rows(get(p + f"self_attn.{n}_proj.weight"), r, tp) for n in "qkv")
            layer.attn.qkv = _p(torch.cat([q, k, v]).contiguous())
            layer.attn.o = _p(shard_cols(get(p + "self_attn.o_proj.weight"), r, tp).contiguous())
            layer.ln1 = _p(get(p + "input_layernorm.weight"))
            layer.ln2 = _p(get(p + "post_attention_layernorm.weight"))
            self._load_mlp_hf(i, layer.mlp, get, p)
        return self

    def _load_mlp_hf(self, i, mlp, get, p) -> None:
        tp, r = self.st.tp_size, self.st.tp_rank
        g = shard_rows(get(p + "mlp.gate_proj.weight"), r, tp)
        u = shard_rows(get(p + "mlp.up_proj.weight"), r, tp)
        mlp.gate_up = _p(gemm.interleave_gate_up(g, u).contiguous())
        mlp.down = _p(shard_cols(get(p + "mlp.down_proj.weight"), r, tp).contiguous())

    def hf_state_dict(self) -> dict:
        """Weights under HF Llama/Mixtral names (unfused q/k/v, gate/up; TP=1 only)."""
        assert self.st.tp_size == 1, "export a TP=1 model"
        cfg = self.cfg
        q_sz, kv_sz = cfg.q_size, cfg.kv_size
        out = {"model.embed_tokens.weight": self.embed[:cfg.vocab_size], "model.norm.weight": self.norm}
        if self.lm_head is not self.embed:
            out["lm_head.weight"] = self.lm_head[:cfg.vocab_size]
        for i, layer in enumerate(self.layers):
            p = f"model.layers.{i}."
            q, k, v = layer.attn.qkv.split([q_sz, kv_sz, kv_sz])
            out.update({p + "self_attn.q_proj.weight": q, p + "self_attn.k_proj.weight": k,
                        p + "self_attn.v_proj.weight": v, p + "self_attn.o_proj.weight": layer.attn.o,
                        p + "input_layernorm.weight": layer.ln1, p + "post_attention_layernorm.weight": layer.ln2})
            out.update(self._mlp_hf_state(p, layer.mlp))
        return {k: v.detach().contiguous().cpu() for k, v in out.items()}

    def _mlp_hf_state(self, p: str, mlp) -> dict:
        g, u = gemm.deinterleave_gate_up(mlp.gate_up)
        return {p + "mlp.gate_proj.weight": g, p + "mlp.up_proj.weight": u, p + "mlp.down_proj.weight": mlp.down}

    def save_hf(self, path: str) -> None:
        """Write ``config.json`` + ``model.safetensors`` (checkpoint / export; reload with ``load_hf``)."""
        import json
        import os

        from safetensors.torch import save_file
        os.makedirs(path, exist_ok=True)
        cfg = self.cfg
        hf = {"architectures": ["MixtralForCausalLM" if cfg.is_moe else "LlamaForCausalLM"],
              "vocab_size": cfg.vocab_size, "hidden_size": cfg.hidden_size,
              "intermediate_size": cfg.intermediate_size, "num_hidden_layers": cfg.num_layers,
              "num_attention_heads": cfg.num_heads, "num_key_value_heads": cfg.num_kv_heads,
              "head_dim": cfg.head_dim, "rope_theta": cfg.rope_theta, "rms_norm_eps": cfg.rms_eps,
              "max_position_embeddings": cfg.max_position, "tie_word_embeddings": cfg.tie_embeddings,
              "bos_token_id": cfg.bos_token_id, "eos_token_id": cfg.eos_token_id, "_name_or_path": cfg.name}
        if cfg.is_moe:
            hf.update(num_local_experts=cfg.num_experts, num_experts_per_tok=cfg.experts_per_token)
        if cfg.rope_scaling:
            hf["rope_scaling"] = cfg.rope_scaling
        with open(os.path.join(path, "config.json"), "w") as f:
            json.dump(hf, f, indent=1)
        save_file(self.hf_state_dict(), os.path.join(path, "model.safetensors"))

    # ------------------------------------------------------------------ forward
    def embed_tokens(self, ids: torch.Tensor) -> torch.Tensor:
        """Vocab-parallel embedding: one gather kernel with the out-of-shard mask fused
        (``ops.embedding``), then the TP all-reduce assembles the rows."""
        start = self.vocab_start if self.st.tp_size > 1 else 0
        x = ops.embedding(ids, self.embed, start, self.embed.shape[0] if self.st.tp_size == 1 else self.vocab_local)
        return comm.tp_all_reduce(x) if self.st.tp_size > 1 else x

    def forward(self, input_ids: torch.Tensor, positions: torch.Tensor, md: attn_ops.AttnMetadata,
                kv_caches: List[Tuple[torch.Tensor, torch.Tensor]]) -> torch.Tensor:
        """Returns the final-normed hidden states [T, H]."""
        if self._sp_ok(input_ids):
            return self._forward_sp(input_ids, positions, md, kv_caches)
        x = self.embed_tokens(input_ids)
        ws = self.workspace(x.shape[0])
        # the folded chain serves decode batches up to DECODE_MAX_M rows; steps carrying prefill
        # chunks above 64 rows keep the library GEMMs (hipBLASLt) of the general path
        if ws is not None and (md.num_prefill == 0 or x.shape[0] <= gemm.SKINNY_MAX_M) and self._rowscale_ok(x):
            return self._forward_rowscale(x, positions, md, kv_caches, ws)
        residual = None
        for i, layer in enumerate(self.layers):
            if residual is None:
                residual = x
                x = ops.rms_norm(x, layer.ln1, layer.eps)
            else:
                x, residual = add_norm(x, residual, layer.ln1, layer.eps)
            x = layer.attn(x, positions, md, self.cos_sin, kv_caches[i], ws)
            x, residual = self._mlp_block(layer, x, residual, ws)
        x, _ = add_norm(x, residual, self.norm, self.cfg.rms_eps)
        return x

    def _mlp_block(self, layer, x, residual, ws):
        """post-attention residual add + RMSNorm, then the MLP (its output may be pending)."""
        x, residual = add_norm(x, residual, layer.ln2, layer.eps)
        return layer.mlp(x, ws), residual

    # ------------------------------------------------------------------ sequence parallel (TP prefill)
    def _sp_ok(self, ids: torch.Tensor) -> bool:
        return SEQUENCE_PARALLEL and self.st.tp_size > 1 and ids.shape[0] >= SP_MIN_TOKENS

    def _forward_sp(self, input_ids: torch.Tensor, positions: torch.Tensor, md: attn_ops.AttnMetadata,
                    kv_caches: List[Tuple[torch.Tensor, torch.Tensor]]) -> torch.Tensor:
        """TP prefill with a token-sharded residual stream (:mod:`..parallel.comm` SP layout).
        The vocab-parallel embedding partial is reduce-scattered straight into the shard; then
        per layer:

            all-gather(h) -> QKV GEMM (chunk-overlapped) -> attention -> o GEMM -> reduce-scatter
            residual add + RMSNorm on the shard
            all-gather(h) -> gate_up + SiLU -> down GEMM -> reduce-scatter
            residual add + RMSNorm on the shard

        and the final-normed shard is all-gathered for the LM head."""
        T = input_ids.shape[0]
        chunks = comm.overlap_chunks(T) if input_ids.is_cuda else 1
        lay = comm.SPLayout(T, chunks)
        emb = ops.embedding(input_ids, self.embed, self.vocab_start, self.vocab_local)
        residual = comm.sp_reduce_scatter(emb, lay)
        del emb
        h = ops.rms_norm(residual, self.layers[0].ln1, self.layers[0].eps)
        for i, layer in enumerate(self.layers):
            at = layer.attn
            qkv = comm.sp_all_gather(h, lay, comm.RowsFn(
                lambda r, o, w=at.qkv, wp=at.qkv_p: gemm.linear(r, w, out=o, packed=wp), at.qkv.shape[0]))
            a = at.drop(at.attend(qkv, positions, md, self.cos_sin, kv_caches[i]))
            del qkv
            o = comm.sp_reduce_scatter(a, lay, comm.RowsFn(
                lambda r, out, w=at.o, wp=at.o_p: gemm.linear(r, w, out=out, packed=wp), at.o.shape[0]))
            h, residual = ops.fused_add_rms_norm(o, residual, layer.ln2, layer.eps)
            m = self._sp_mlp(layer, h, lay)
            nxt = self.layers[i + 1].ln1 if i + 1 < len(self.layers) else self.norm
            h, residual = ops.fused_add_rms_norm(m, residual, nxt, layer.eps)
        return comm.sp_all_gather(h, lay)

    def _sp_mlp(self, layer, h: torch.Tensor, lay) -> torch.Tensor:
        """Dense MLP on the SP shard: all-gather → gate_up + SiLU → down → reduce-scatter."""
        mlp = layer.mlp
        g = comm.sp_all_gather(h, lay, comm.RowsFn(
            lambda r, o, w=mlp.gate_up, wp=mlp.gate_up_p: o.copy_(gemm.linear_silu(r, w, packed=wp))
            if w.is_meta else gemm.silu_and_mul_interleaved(gemm.linear(r, w), out=o), mlp.gate_up.shape[0] // 2))
        return comm.sp_reduce_scatter(g, lay, comm.RowsFn(
            lambda r, o, w=mlp.down, wp=mlp.down_p: gemm.linear(r, w, out=o, packed=wp), mlp.down.shape[0]))

    # ------------------------------------------------------------------ folded-norm decode chain
    def _rowscale_ok(self, x: torch.Tensor) -> bool:
        l0 = self.layers[0]
        if self.st.tp_size > 1:
            # TP: every row-parallel projection ends in the fused IPC collective (slab reduce +
            # xGMI peer sum + residual add + norm parts in one launch)
            car = self.st.custom_ar
            if car is None or not car.supports_reduce_residual(x.shape[0], self.cfg.hidden_size):
                return False
        return (l0.attn.qkv_pf is not None and getattr(l0.mlp, "gate_up_pf", None) is not None
                and self.cfg.hidden_size % 1024 == 0 and gemm.norm_fusable(self.cfg.hidden_size)
                and gemm.skinny_ok(x, l0.attn.qkv, max_m=gemm.DECODE_MAX_M))

    def _forward_rowscale(self, x: torch.Tensor, positions: torch.Tensor, md: attn_ops.AttnMetadata,
                          kv_caches: List[Tuple[torch.Tensor, torch.Tensor]], ws: torch.Tensor) -> torch.Tensor:
        """Decode step with the RMSNorms folded into the projections (FOLD_NORM):

            qkv  = rinv1 * (residual @ (Wqkv diag ln1)^T)   split-K slabs -> attention (RoPE, cache)
            residual += o-proj(attn)                        + per-row sums of squares (parts)
            h    = silu / mul of rinv2 * (residual @ (Wgu diag ln2)^T)
            residual += down(h)                             + parts for the next layer's rinv1

        rinv = rsqrt(mean(residual^2) + eps) is formed by each consumer from the parts."""
        T, H = x.shape
        if getattr(self, "_parts_buf", None) is None:
            self._parts_buf = torch.zeros((H // 64) * gemm.DECODE_MAX_M, dtype=torch.float32, device=self.device)
            self._parts_buf2 = torch.zeros_like(self._parts_buf)
        buf, buf2 = self._parts_buf, self._parts_buf2
        residual = x
        if self.st.tp_size > 1:
            parts = gemm.residual_parts(None, residual, buf)
            return self._forward_rowscale_tp(residual, parts, positions, md, kv_caches, ws, buf, buf2)
        pending = None  # the previous layer's down slabs, not yet added to the residual
        for i, layer in enumerate(self.layers):
            parts = gemm.residual_parts(pending, residual, buf)
            a = self._decode_attn(layer, residual, parts, positions, md, kv_caches[i], ws)
            # o-projection slabs from 64-row n-blocks at half the split (-0.7..1.5 % decode step,
            # profiles/r2_decode_ab.txt: fewer fp32 slab bytes written and re-read); the residual
            # update inside the O launch (1 % slower, profiles/r4_o_inlaunch_ab.jsonl) and as phase 0
            # of the fused launches (3 % slower, profiles/r5_phase_ab.jsonl) were removed in round 6
            o = gemm.linear_partial(a, layer.attn.o, ws, packed=layer.attn.o_p, half=True)
            parts = gemm.residual_parts(o, residual, buf2)
            pending = self._decode_mlp(layer, residual, parts, ws)
        x, _ = gemm.partial_add_rms_norm(pending, residual, self.norm, self.cfg.rms_eps)
        return x

    def _qkv_attn_fused_ok(self, at, T: int, nparts: int, md) -> bool:
        # (a TP rank sharing its GPU keeps the two launches: a hand-off lost to a co-tenant has a
        # fallback only at TP = 1 -- a TP group cannot re-run one rank's step, llm_engine.py)
        return (md.num_prefill == 0 and gemm.QKV_ATTN_FUSED and at.nkv >= gemm.QKV_ATTN_MIN_KV
                and gemm.fused_rows_ok(T, nparts) and md.num_decode == T
                and not (self.st.shared_device and self.st.tp_size > 1))

    def _decode_attn(self, layer, residual: torch.Tensor, parts: torch.Tensor, positions: torch.Tensor,
                     md: attn_ops.AttnMetadata, kv: Tuple[torch.Tensor, torch.Tensor], ws: torch.Tensor):
        """Folded-norm QKV projection + RoPE + KV write + attention of one layer -> [T, nq * 128]."""
        at = layer.attn
        kc, vc = kv
        T = residual.shape[0]
        rs = gemm.RowScale(parts, layer.eps)
        if self._qkv_attn_fused_ok(at, T, parts.shape[0], md):
            # QKV slabs handed to the decode attention in-launch (one launch, csrc/kernels/decode_fused.hip);
            # deadlock-free on a shared GPU too: the QKV tiles never wait and dispatch first
            return gemm.qkv_attn_fused(residual, at.qkv_pf, rs, ws, positions, self.cos_sin, kc, vc, md, at.scale,
                                       at.nq, at.nkv, self._flow_qkv)
        # (64-row n-blocks at half the split: half the slabs the attention prologue sums -- the 70B
        # TP=8 shard's 10 n-blocks otherwise take split 16; one 64-row tile only: the row-tiled wide
        # batches keep 128-row n-blocks, 8B at 256 rows 34.5 vs 26 us, profiles/r5_wide_256_kgrid.md)
        p = gemm.linear_partial_rowscale(residual, at.qkv, ws, rs, packed=at.qkv_pf,
                                         half=gemm.QKV_HALF and T <= gemm.SKINNY_MAX_M)
        if md.num_prefill == 0:
            return attn_ops.paged_decode_from_qkv(p, positions, self.cos_sin, kc, vc, md, at.scale, at.nq, at.nkv)
        q = gemm.qkv_reduce_rope_cache(p, positions, self.cos_sin, kc, vc, md.slot_mapping, at.nq, at.nkv)
        return attn_ops.paged_attention(q, kc, vc, md, at.scale)

    def _decode_mlp(self, layer, residual: torch.Tensor, parts: torch.Tensor, ws: torch.Tensor) -> gemm.Partial:
        """Folded-norm gate_up + SiLU and the down projection of one layer -> down's split-K slabs."""
        mlp = layer.mlp
        rs = gemm.RowScale(parts, layer.eps)
        if gemm.mlp_fused_ok(residual, mlp.gate_up_pf, mlp.down_p, parts.shape[0]) and not self.st.shared_device:
            # gate_up + SiLU and the down slabs in one launch (down's launch ramp hidden)
            return gemm.mlp_fused(residual, mlp.gate_up_pf, mlp.down_p, rs, ws, self._flow)
        h = self._decode_gate_up(layer, residual, parts)
        return gemm.linear_down(h, mlp.down, ws, mlp.down_p)  # tiled as the fused launch tiles it

    def _decode_gate_up(self, layer, residual: torch.Tensor, parts: torch.Tensor) -> torch.Tensor:
        """Folded-norm gate_up + SiLU of the two-launch decode MLP -> h [T, I] bf16."""
        mlp = layer.mlp
        rs = gemm.RowScale(parts, layer.eps)
        if _wide_mfma_ok(residual, mlp.gate_up_pf):
            # rows * folded block-packed weight (ln2 inside): normalise with unit weights
            x = gemm.norm_apply(residual, parts, self._ones_h, layer.eps)
            return gemm_prefill.linear(x, mlp.gate_up, silu=True, packed=mlp.gate_up_pf)
        if residual.shape[0] > GATE_UP_SKINNY_MAX_M and not mlp.gate_up.is_meta:
            # hipBLASLt's MFMA GEMM wins on the 235 MB gate_up above 192 rows (67 vs 85 us at 256,
            # 97 vs 155 at 512: profiles/r4_wide_decode_probe.jsonl) even with the norm and SiLU as
            # separate kernels
            x = gemm.norm_apply(residual, parts, layer.ln2, layer.eps)
            return gemm.silu_and_mul_interleaved(F.linear(x, mlp.gate_up))
        # split over K like the fused launch's gate_up when its n-blocks cannot fill the chip
        return gemm.linear_silu(residual, mlp.gate_up, ws=self._ws_gu, packed=mlp.gate_up_pf, rowscale=rs)

    def _forward_rowscale_tp(self, residual: torch.Tensor, parts: torch.Tensor, positions: torch.Tensor,
                             md: attn_ops.AttnMetadata, kv_caches: List[Tuple[torch.Tensor, torch.Tensor]],
                             ws: torch.Tensor, buf: torch.Tensor, buf2: torch.Tensor) -> torch.Tensor:
        """TP decode step of the folded-norm chain, per layer (the TP=1 chain's launches with the
        residual updates replaced by the fused collective):

            a     = qkv_attn_fused: rinv1 * (residual @ (Wqkv_local diag ln1)^T) split-K slabs
                    handed in-launch to the decode attention (RoPE, KV write)
            o     = split-K slabs of a @ Wo_local^T  -> fused collective: slab sum, xGMI peer
                    sum, residual += , norm parts (parallel/custom_ar.py reduce_residual)
            d     = mlp_fused: silu / mul of rinv2 * (residual @ (Wgu_local diag ln2)^T) (split
                    over K: 56 n-blocks at 70B TP=8) handed in-launch to the down slabs
                  -> fused collective

        Each row-parallel projection costs its GEMM and ONE collective launch (2 x 80
        all-reduces per 70B TP=8 step).  Launches per layer: 6 with the fused QKV -> attention and MLP
        launches (8B-like shards: >= 4 kv heads per rank), 8 at the 70B TP=8 shard (one kv head: QKV |
        attention; gate_up split over K: gate_up | SiLU reduce | down), profiles/r5_decode_attention.md
        -- 6 there too when the collectives ride in their consumers' launches (_forward_tp_carried)."""
        car = self.st.custom_ar
        if self._carry_ok(residual, md):
            return self._forward_tp_carried(residual, parts, positions, md, kv_caches, ws, buf, buf2)
        for i, layer in enumerate(self.layers):
            at, mlp = layer.attn, layer.mlp
            a = self._decode_attn(layer, residual, parts, positions, md, kv_caches[i], ws)
            parts = self._tp_row_collective(at.drop(a), at.o, at.o_p, ws, residual, buf2)
            if gemm.mlp_fused_ok(residual, mlp.gate_up_pf, mlp.down_p, parts.shape[0]) and not self.st.shared_device:
                parts = car.reduce_residual(self._decode_mlp(layer, residual, parts, ws), residual, buf)
            else:
                h = self._decode_gate_up(layer, residual, parts)
                parts = self._tp_row_collective(h, mlp.down, mlp.down_p, ws, residual, buf, down=True)
        return gemm.norm_apply(residual, parts, self.norm, self.cfg.rms_eps)

    # the TP decode collectives carried by the launch of the projection that consumes them
    # (kernels/car_gemm.hip); None: POLYKEY_TP_CARRY, off on a shared GPU.  Default OFF: on the
    # loopback group the carried chain is bit-identical but 0.12 ms per 70B TP=8 rank step slower
    # (7.58 vs 7.45 ms, profiles/r6_carry.md): the consumer's A operand, written in-launch by other
    # XCDs, must be read past the (per-XCD, non-coherent) L2 -- the 56 n-blocks of a split re-read it
    # from the Infinity Cache instead of L2 -- which costs more than the launch boundary it saves.
    # Kept for the 8-GPU A/B, where the xGMI exchange is longer than loopback's.  Per site
    # (profiles/r6_carry.md kernel table): the o -> gate_up launch is at parity with its two plain
    # launches (35.5 vs 35.8 us), the down -> QKV one 2 us slower (21.3 vs 19.3 us: 160 QKV tiles
    # wait on the whole collective for the row scale) -- POLYKEY_TP_CARRY=gate_up carries only the
    # first.  carry_qkv None: from that variable.
    carry_collectives: Optional[bool] = None
    carry_qkv: Optional[bool] = None

    def _carry_ok(self, residual: torch.Tensor, md) -> bool:
        """The carried chain (:meth:`_forward_tp_carried`) takes pure-decode steps of one 64-row tile
        on the two-shot collective (TP = 4 / 8), for shards whose gate_up is split over K (no fused
        MLP launch) and whose QKV is not fused with the attention (70B TP=8: one kv head per rank).
        Ranks sharing a GPU keep the plain chain: a rank's consumer tiles wait inside a launch for
        its collective, whose peers' workgroups need slots on the same device."""
        on = self.carry_collectives
        if on is None:
            on = os.environ.get("POLYKEY_TP_CARRY", "0") in ("1", "gate_up") and not self.st.shared_device
        car = self.st.custom_ar
        M, H = residual.shape
        l0 = self.layers[0]
        return bool(on and residual.is_cuda and md.num_prefill == 0 and md.num_decode == M
                    and hasattr(car, "carry_ok") and car.carry_ok(M, H) and not gemm.TP_PUSH
                    and gemm.TP_DECODE_CHUNKS < 2 and isinstance(l0.mlp, LlamaMLP)
                    and not gemm.mlp_fused_ok(residual, l0.mlp.gate_up_pf, l0.mlp.down_p, H // 256)
                    and gemm.gate_up_split(l0.mlp.gate_up.shape[0], H, M) > 1
                    and not self._qkv_attn_fused_ok(l0.attn, M, H // 256, md)
                    and getattr(self, "_ws_gu", None) is not None)

    def _forward_tp_carried(self, residual: torch.Tensor, parts: torch.Tensor, positions: torch.Tensor,
                            md: attn_ops.AttnMetadata, kv_caches: List[Tuple[torch.Tensor, torch.Tensor]],
                            ws: torch.Tensor, buf: torch.Tensor, buf2: torch.Tensor) -> torch.Tensor:
        """The TP decode chain with every collective but the last carried by its consumer's launch
        (gemm.linear_partial_rowscale_car), per layer:

            attention from the QKV slabs (RoPE, KV write)            [QKV came with the last launch]
            o     = split-K slabs of a @ Wo_local^T
            [collective(o) -> residual, parts | gate_up slabs of rinv2 * residual @ Wgu'^T]  ONE launch
            h     = SiLU reduce of the gate_up slabs
            d     = split-K slabs of h @ Wdown_local^T
            [collective(d) -> residual, parts | next layer's QKV slabs]                     ONE launch

        6 launches per 70B TP=8 layer instead of 8; bit-identical to the plain chain (the same
        collective, the same consumer tiling, the row scale applied after accumulation)."""
        car = self.st.custom_ar
        dev = car.device_ctx()
        if getattr(self, "_flow_car", None) is None:
            self._flow_car = torch.zeros(gemm.FLOW_WORDS, dtype=torch.int32, device=self.device)
        flow = self._flow_car
        M, H = residual.shape
        qkv_half = gemm.QKV_HALF and M <= gemm.SKINNY_MAX_M
        carry_qkv = self.carry_qkv
        if carry_qkv is None:
            carry_qkv = os.environ.get("POLYKEY_TP_CARRY", "0") != "gate_up"
        L = len(self.layers)
        qkv = None  # this layer's QKV slabs when the previous launch produced them
        for i, layer in enumerate(self.layers):
            at, mlp = layer.attn, layer.mlp
            kc, vc = kv_caches[i]
            if qkv is None:
                a = self._decode_attn(layer, residual, parts, positions, md, kv_caches[i], ws)
            else:
                a = attn_ops.paged_decode_from_qkv(qkv, positions, self.cos_sin, kc, vc, md, at.scale, at.nq, at.nkv)
            o = gemm.linear_partial(at.drop(a), at.o, ws, packed=at.o_p, half=True)
            N2 = mlp.gate_up.shape[0]
            parts, gu = gemm.linear_partial_rowscale_car(dev, o, residual, buf2, mlp.gate_up, self._ws_gu, layer.eps,
                                                         flow, packed=mlp.gate_up_pf, S=gemm.gate_up_split(N2, H, M))
            h = torch.empty((M, N2 // 2), dtype=residual.dtype, device=residual.device)
            gemm.silu_reduce(gu, h)
            d = gemm.linear_down(h, mlp.down, ws, mlp.down_p)
            if i + 1 < L and carry_qkv:
                nxt = self.layers[i + 1]
                parts, qkv = gemm.linear_partial_rowscale_car(dev, d, residual, buf, nxt.attn.qkv, ws, nxt.eps, flow,
                                                              packed=nxt.attn.qkv_pf, half=qkv_half)
            else:
                parts, qkv = car.reduce_residual(d, residual, buf), None
        return gemm.norm_apply(residual, parts, self.norm, self.cfg.rms_eps)

    def _tp_row_collective(self, x: torch.Tensor, w: torch.Tensor, wp: Optional[torch.Tensor], ws: torch.Tensor,
                           residual: torch.Tensor, buf: torch.Tensor, down: bool = False) -> torch.Tensor:
        """A row-parallel decode projection x @ w^T + its fused TP collective (custom_ar
        reduce_residual: slab sum, xGMI exchange, residual add, norm parts) -> the parts.

        With gemm.TP_DECODE_CHUNKS = C > 1 the projection runs as C column-chunk GEMMs on the
        compute stream (w's packed rows are n-block-major, so a chunk is a contiguous row range);
        after each, an event forks the chunk's collective onto the comm stream, so the xGMI
        exchange of chunk c runs while the compute stream computes chunk c + 1 (SURVEY.md §2.3 /
        BASELINE.json:5: all-reduce over xGMI overlapped with the GEMMs on HIP streams).  Every
        collective waits only on a finished GEMM: no in-kernel wait on a producer that a shared
        hardware queue could order behind it.  The compute stream joins before the residual's next
        reader.  ``down``: tiled as gemm.linear_down (else linear_partial, half)."""
        car = self.st.custom_ar
        M, N = residual.shape
        if (gemm.TP_PUSH and wp is not None and residual.is_cuda and hasattr(car, "push_ok")
                and getattr(self, "_push_counters", None) is not None and car.push_ok(M, N, 64)):
            # the GEMM's epilogue stores each finished tile into its owner's slot (xGMI under the
            # GEMM's tail); the collective starts at the reduce-scatter
            nbc = gemm.push_projection(x, w, ws, wp, self._push_counters, car.push_target(), down=down)
            self._push_calls = getattr(self, "_push_calls", 0) + 1  # tools/tp_rehearsal.py reports it
            return car.reduce_residual_pushed(residual, buf, nbc)

        def gemm_of(xx, ww, pp, out):
            return gemm.linear_down(xx, ww, out, pp) if down else gemm.linear_partial(xx, ww, out, packed=pp, half=True)
        C = gemm.TP_DECODE_CHUNKS
        if (C < 2 or wp is None or not residual.is_cuda or not hasattr(car, "reduce_residual_chunk")
                or M > gemm.FUSED_MAX_M or (N // C) % 128 or not car.chunks_ok(M, N, C)
                or not self._overlap_streams_ok()):
            return car.reduce_residual(gemm_of(x, w, wp, ws), residual, buf)
        Nc = N // C
        K = x.shape[1]
        S_c = gemm.choose_split(Nc, K, M) if down else max(1, gemm.choose_split(Nc, K, M) // 2)
        if ws.numel() < C * S_c * M * Nc:  # the chunks' slabs side by side in the workspace
            return car.reduce_residual(gemm_of(x, w, wp, ws), residual, buf)
        main = torch.cuda.current_stream(residual.device)
        cs = comm.comm_stream(residual.device)
        off = 0
        for c in range(C):
            rows = slice(c * Nc, (c + 1) * Nc)
            p = gemm_of(x, w[rows], wp[rows], ws[off:])
            off += p.S * M * Nc
            ev = torch.cuda.Event()
            ev.record(main)
            cs.wait_event(ev)
            with torch.cuda.stream(cs):
                car.reduce_residual_chunk(p, residual, buf, c, C)
        main.wait_stream(cs)
        return buf.view(-1)[: car.nparts(M, N) * M].view(-1, M)

    # the chunked TP decode chain regardless of _overlap_streams_ok (tests: 8 ranks on one GPU)
    force_overlap_streams = False

    def _overlap_streams_ok(self) -> bool:
        """The overlapped TP chain forks a comm stream inside the captured decode graph.  It can only
        pay where the two streams really run concurrently: one rank per GPU and at least two hardware
        queues per process.  (The round-5 crash in ``graph.replay`` under one hardware queue,
        profiles/r5_tp_overlap.md §1, belonged to the removed design whose collective kernel spun
        on flags of a GEMM queued behind it; the chunked design never waits in-kernel on a producer,
        so one queue only serialises it -- gated off because it then only adds launches.)"""
        if self.force_overlap_streams:
            return True
        return not self.st.shared_device and int(os.environ.get("GPU_MAX_HW_QUEUES", "4")) >= 2

    def workspace(self, M: int) -> Optional[torch.Tensor]:
        """fp32 split-K slab buffer for decode-sized batches (fixed address: graph-safe)."""
        if self.device.type != "cuda" or M > gemm.DECODE_MAX_M:
            return None
        if getattr(self, "_ws", None) is None:
            self._ws = torch.empty(self._workspace_elems(), dtype=torch.float32, device=self.device)
            # hand-off tickets of the fused decode MLP launch (gemm.mlp_fused), left zeroed by every launch
            self._flow = torch.zeros(gemm.FLOW_WORDS, dtype=torch.int32, device=self.device)
            gemm.fused_err_word()  # before the first fused launch (engine polls gemm.check_fused)
            self._flow_qkv = torch.zeros(gemm.FLOW_WORDS, dtype=torch.int32, device=self.device)
            # slabs of a gate_up split over K (gemm.gate_up_split > 1: the 70B TP=8 shard)
            n = self._gate_up_split_elems()
            self._ws_gu = torch.empty(n, dtype=torch.float32, device=self.device) if n else None
            # split-K arrival counters of the push GEMMs (gemm.TP_PUSH: o / down, N = hidden)
            self._push_counters = (torch.zeros(self.cfg.hidden_size // 64, dtype=torch.int32, device=self.device)
                                   if self.st.tp_size > 1 else None)
        return self._ws

    def _gate_up_split_elems(self) -> int:
        gu = getattr(self.layers[0].mlp, "gate_up", None)
        if gu is None or gu.dim() != 2:
            return 0
        N2, K = gu.shape
        splits = [(gemm.gate_up_split(N2, K, M), M) for M in range(1, gemm.FUSED_MAX_M + 1)]
        return max(sg * M * N2 for sg, M in splits) if any(sg > 1 for sg, _ in splits) else 0

    def _workspace_elems(self) -> int:
        shapes = []
        l0 = self.layers[0]
        for w in (l0.attn.qkv, l0.attn.o) + self._mlp_weights(l0.mlp):
            if w is not None:  # the split shrinks as row tiles grow: take the largest S * M
                shapes.append(max(gemm.choose_split(w.shape[0], w.shape[1], M) * M
                                  for M in range(1, gemm.DECODE_MAX_M + 1)) * w.shape[0])
        return max(shapes + [1])

    def _mlp_weights(self, mlp) -> tuple:
        return (mlp.gate_up, mlp.down)

    def pack_decode_weights(self, mode: Optional[str] = None) -> bool:
        """Give every dense projection and the LM head a block-packed copy
        (:func:`gemm.pack_weight`) for the decode GEMM, which streams it faster than row-major
        (tools/bench_gemm.py, tools/gemm_lab.hip).  Prefill keeps using the row-major weight
        through hipBLASLt, so this doubles projection memory: ``auto`` packs when both copies fit
        in 75 % of this rank's share of HBM (8B: +16 GB of 288 GB; Mixtral-8x7B: +90 GB; ranks
        sharing one GPU split it).  When they do not (70B on one GPU, an 8-rank TP=8 rehearsal on
        one GPU) the projections are kept ONLY packed: prefill then reads the same layout through
        the hand-written MFMA GEMM (``csrc/kernels/gemm_prefill.hip``) and the row-major
        attributes become shape-only (meta) placeholders.  With folded norms (Llama MLP) the
        packed-only copies of QKV and gate/up carry their RMSNorm weight, and prefill normalises
        with unit weights (``ln1`` / ``ln2`` become ones; the originals stay as ``ln*_folded``).
        ``POLYKEY_PACKED_WEIGHTS`` = auto | 1 (both copies) | packed (packed only) | 0."""
        mode = mode or os.environ.get("POLYKEY_PACKED_WEIGHTS", "auto")
        if mode == "0" or self.device.type != "cuda" or not gemm.SKINNY_ENABLED:
            return False
        head_bytes = self.lm_head.numel() * self.lm_head.element_size()
        packed_only = mode == "packed"
        if mode == "auto":
            total = torch.cuda.get_device_properties(self.device).total_memory / max(1, self.st.ranks_per_device)
            proj = sum(w.numel() * w.element_size() for w in self.layers.parameters())
            if 2 * proj + 2 * head_bytes > 0.75 * total:
                packed_only = True
        if packed_only and not self._packed_prefill_ok():
            return False
        fold = FOLD_NORM and isinstance(self.layers[0].mlp, LlamaMLP)

        def pack(owner, name: str, dst: str, w: Optional[torch.Tensor] = None) -> None:
            src = getattr(owner, name)
            setattr(owner, dst, gemm.pack_weight(src if w is None else w))
            if packed_only:  # free the row-major copy now: peak memory is one projection over
                setattr(owner, name, _p(torch.empty(src.shape, dtype=src.dtype, device="meta")))

        for layer in self.layers:
            if fold:
                layer.attn.qkv_pf = pack_folded(layer.attn, "qkv", layer.ln1, packed_only)
                layer.mlp.gate_up_pf = pack_folded(layer.mlp, "gate_up", layer.ln2, packed_only)
                if packed_only:  # prefill reads the folded copies: normalise with unit weights
                    layer.attn.qkv_p, layer.mlp.gate_up_p = layer.attn.qkv_pf, layer.mlp.gate_up_pf
                    layer.ln1_folded, layer.ln2_folded = layer.ln1, layer.ln2
                    layer.ln1 = _p(torch.ones_like(layer.ln1))
                    layer.ln2 = _p(torch.ones_like(layer.ln2))
                pack(layer.mlp, "down", "down_p")
            else:
                pack(layer.attn, "qkv", "qkv_p")
                if isinstance(layer.mlp, LlamaMLP):
                    pack(layer.mlp, "gate_up", "gate_up_p")
                    pack(layer.mlp, "down", "down_p")
                else:
                    self._pack_mlp(layer.mlp)
            pack(layer.attn, "o", "o_p")
        if self.lm_head.shape[0] % 128 == 0 and self.lm_head.shape[1] % 256 == 0:
            self.lm_head_p = gemm.pack_weight(self.lm_head)
        self.packed_only = packed_only
        self._ones_h = torch.ones(self.cfg.hidden_size, dtype=self.lm_head.dtype, device=self.device)
        return True

    def _packed_prefill_ok(self) -> bool:
        """Every dense projection is a shape the packed-W prefill GEMM tiles (Llama MLP; per-rank
        shapes under TP, e.g. 70B TP=8: QKV 1280 x 8192, o 8192 x 1024, gate/up 7168 x 8192,
        down 8192 x 3584)."""
        from ..ops import gemm_prefill
        l0 = self.layers[0]
        if not isinstance(l0.mlp, LlamaMLP):
            return False
        return all(gemm_prefill.supported(w.shape[0], w.shape[1]) and w.shape[1] % 128 == 0
                   for w in (l0.attn.qkv, l0.attn.o, l0.mlp.gate_up, l0.mlp.down))

    def _pack_mlp(self, mlp) -> None:
        mlp.gate_up_p = gemm.pack_weight(mlp.gate_up)
        mlp.down_p = gemm.pack_weight(mlp.down)

    def compute_logits(self, hidden: torch.Tensor) -> torch.Tensor:
        """hidden [B, H] → logits [B, vocab] (bf16; all-gathered across TP)."""
        # decode: the skinny kernel streams the block-packed vocab projection with non-temporal
        # loads (1 GB for Llama-3: 179 us vs hipBLASLt's 198-208 us, tools/gemm_lab.hip)
        # above 128 rows hipBLASLt's MFMA GEMM is the faster one (tools/bench_gemm_rows.py, 8B:
        # 284 vs 358 us at 256 rows, 492 vs 668 at 512; profiles/r3_decode_rows.txt)
        wp = getattr(self, "lm_head_p", None)
        if hidden.shape[0] > LM_HEAD_SKINNY_MAX_M and _wide_mfma_ok(hidden, wp):
            logits = gemm_prefill.linear(hidden, self.lm_head, packed=wp)
        elif wp is not None and gemm.skinny_ok(hidden, self.lm_head, max_m=gemm.DECODE_MAX_M) and (
                hidden.shape[0] <= LM_HEAD_SKINNY_MAX_M or self.lm_head.is_meta):
            logits = gemm.linear(hidden, self.lm_head, packed=wp, max_m=gemm.DECODE_MAX_M)
        else:
            logits = F.linear(hidden, self.lm_head)
        logits = comm.tp_all_gather_last(logits)
        if logits.shape[-1] != self.cfg.vocab_size:
            logits = logits[..., :self.cfg.vocab_size]
        return logits
