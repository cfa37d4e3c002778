"""Mixtral-8x7B: Llama attention + sparse top-2 MoE MLP (config 5 of BASELINE.json).

Expert placement on a TP group of size ``tp``:

* ``ep == 1``  — every rank holds all 8 experts with the intermediate dim sharded by ``tp``
  (tensor-parallel experts; output all-reduced like the dense MLP);
* ``ep == tp`` — expert parallel: rank r holds experts ``[r*E/ep, (r+1)*E/ep)`` unsharded.
  Tokens are already replicated on every rank by the TP attention, so each rank routes all
  tokens, computes only its local experts (a rank whose experts received no token reads no
  expert weights at all) and the combine is one all-reduce;
* ``tp == 1, ep == world`` — DP attention + EP: each rank serves its own requests with a full
  copy of the attention weights and routes its tokens to the experts' owners with the
  all-to-all dispatch / combine of :mod:`..parallel.ep` (ranks step in lockstep; a rank with
  nothing scheduled runs :meth:`MixtralForCausalLM.idle_forward`).

Mixtral bf16 (~93 GB) also fits a single 288 GB MI355X (``tp = ep = 1``).
"""
from __future__ import annotations

from typing import Optional

import torch
from torch import nn

from ..ops import gemm, moe
from ..parallel import comm, ep as ep_comm
from ..parallel.state import get_state
from .llama import LlamaForCausalLM, _p
from .weights import random_shard, shard_cols, shard_rows


class MixtralMoE(nn.Module):
    def __init__(self, num_experts: int, top_k: int, e_lo: int, e_hi: int):
        super().__init__()
        self.E = num_experts
        self.k = top_k
        self.e_lo, self.e_hi = e_lo, e_hi
        self.router = None
        self.w13 = None  # [E_local, 2*I_local, H], gate/up rows interleaved by 16
        self.w2 = None   # [E_local, H, I_local]
        self.w13_p = None  # block-packed decode copies (MixtralForCausalLM._pack_mlp)
        self.w2_p = None

    def forward(self, x: torch.Tensor, ws: Optional[torch.Tensor] = None, routing=None):
        """Combined expert output, or (single rank: nothing to all-reduce) a PendingCombine that
        the next residual add + RMSNorm consumes in one kernel.  ``routing``: (ids, weights)
        from the norm kernel that produced ``x``."""
        st = get_state()
        if st.dp_attention:  # this rank's tokens → their experts' owners and back
            return ep_comm.ep_moe(x, self.router, self.w13, self.w2, self.k, routing=routing, w13_p=self.w13_p,
                                  w2_p=self.w2_p, defer_combine=True)
        single = st.tp_size == 1
        y = moe.fused_moe(x, self.router, self.w13, self.w2, self.k, self.e_lo, self.e_hi, self.w13_p, self.w2_p,
                          defer_combine=single, routing=routing)
        return y if single else comm.tp_all_reduce(y)

    def local(self, x: torch.Tensor) -> torch.Tensor:
        """This rank's unreduced expert output (its experts / its intermediate shard)."""
        return moe.fused_moe(x, self.router, self.w13, self.w2, self.k, self.e_lo, self.e_hi, self.w13_p, self.w2_p)


class MixtralForCausalLM(LlamaForCausalLM):
    def idle_forward(self) -> None:
        """DP attention + EP: a rank with no tokens this step still serves the other ranks' rows
        at every MoE layer (the all-to-alls are collective over the EP group)."""
        x = torch.zeros((0, self.cfg.hidden_size), dtype=self.dtype, device=self.device)
        for layer in self.layers:
            m = layer.mlp
            ep_comm.ep_moe(x, m.router, m.w13, m.w2, m.k, w13_p=m.w13_p, w2_p=m.w2_p)

    def _mlp_block(self, layer, x, residual, ws):
        """Decode (TP = 1, split-K o-projection pending): the residual add + RMSNorm kernel also
        routes every token, so the MoE starts from ready expert ids and weights."""
        if isinstance(x, gemm.Partial) and x.M <= 64 and gemm.norm_fusable(x.N):
            x, residual, ids, w = gemm.partial_add_rms_norm_route(x, residual, layer.ln2, layer.eps, layer.mlp.router,
                                                                   layer.mlp.k)
            return layer.mlp(x, ws, routing=(ids, w)), residual
        return super()._mlp_block(layer, x, residual, ws)

    def _sp_mlp(self, layer, h, lay):
        """Sequence-parallel prefill: every rank routes all tokens of the gathered rows through
        its experts, and the reduce-scatter that returns to the token shard is the combine."""
        return comm.sp_reduce_scatter(layer.mlp.local(comm.sp_all_gather(h, lay)), lay)

    def _make_mlp(self, layer: int) -> nn.Module:
        cfg, st = self.cfg, self.st
        ep = st.ep_size
        per = cfg.num_experts // ep
        e_lo = st.ep_rank * per if ep > 1 else 0
        return MixtralMoE(cfg.num_experts, cfg.experts_per_token, e_lo, e_lo + per)

    def _mlp_weights(self, mlp) -> tuple:
        return ()

    def _init_mlp_random(self, i: int, mlp: MixtralMoE, rows, cols) -> None:
        cfg, st = self.cfg, self.st
        H, I = cfg.hidden_size, cfg.intermediate_size
        tp_shard = st.ep_size == 1 and st.tp_size > 1
        std, seed, dev, dt = cfg.init_std, self._seed, self.device, self.dtype
        # blocks of the logical tensor run along the dim TP shards (rows of w1 / w3, columns of w2)
        full = lambda name, shape, dim=0: random_shard(name, shape, std, seed, dev, dt, 0, 1, dim)
        rstd = cfg.router_init_std if cfg.router_init_std is not None else std
        mlp.router = _p(random_shard(f"l{i}.router", (cfg.num_experts, H), rstd, seed, dev, dt, 0, 1).contiguous())
        w13, w2 = [], []
        for e in range(mlp.e_lo, mlp.e_hi):
            if tp_shard:  # attention TP without EP: every expert sharded Megatron-style
                g, u, d = rows(f"l{i}.e{e}.w1", (I, H)), rows(f"l{i}.e{e}.w3", (I, H)), cols(f"l{i}.e{e}.w2", (H, I))
            else:
                g, u, d = full(f"l{i}.e{e}.w1", (I, H)), full(f"l{i}.e{e}.w3", (I, H)), full(f"l{i}.e{e}.w2", (H, I), 1)
            w13.append(gemm.interleave_gate_up(g, u))
            w2.append(d.contiguous())
        mlp.w13 = _p(torch.stack(w13).contiguous())
        mlp.w2 = _p(torch.stack(w2).contiguous())

    def _pack_mlp(self, mlp) -> None:
        E, N, K = mlp.w13.shape
        mlp.w13_p = gemm.pack_weight(mlp.w13.view(E * N, K)).view(E, N, K)
        E, N, K = mlp.w2.shape
        mlp.w2_p = gemm.pack_weight(mlp.w2.view(E * N, K)).view(E, N, K)

    def _mlp_hf_state(self, p: str, mlp: MixtralMoE) -> dict:
        out = {p + "block_sparse_moe.gate.weight": mlp.router}
        for j, e in enumerate(range(mlp.e_lo, mlp.e_hi)):
            g, u = gemm.deinterleave_gate_up(mlp.w13[j])
            q = p + f"block_sparse_moe.experts.{e}."
            out.update({q + "w1.weight": g, q + "w3.weight": u, q + "w2.weight": mlp.w2[j]})
        return out

    def _load_mlp_hf(self, i, mlp: MixtralMoE, get, p) -> None:
        st = self.st
        tp_shard = st.ep_size == 1 and st.tp_size > 1
        base = p + "block_sparse_moe."
        mlp.router = _p(get(base + "gate.weight").contiguous())
        w13, w2 = [], []
        for e in range(mlp.e_lo, mlp.e_hi):
            g = get(base + f"experts.{e}.w1.weight")
            u = get(base + f"experts.{e}.w3.weight")
            d = get(base + f"experts.{e}.w2.weight")
            if tp_shard:
                g, u, d = shard_rows(g, st.tp_rank, st.tp_size), shard_rows(u, st.tp_rank, st.tp_size), \
                    shard_cols(d, st.tp_rank, st.tp_size)
            w13.append(gemm.interleave_gate_up(g, u))
            w2.append(d.contiguous())
        mlp.w13 = _p(torch.stack(w13).contiguous())
        mlp.w2 = _p(torch.stack(w2).contiguous())
