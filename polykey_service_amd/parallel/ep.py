"""Expert parallelism with all-to-all dispatch / combine (tokens sharded across ranks).

Used when each EP rank holds a *different* slice of tokens (data-parallel attention in front
of the MoE).  Per MoE layer (SURVEY.md §2.3 "Mixtral EP all-to-all"):

1. route local tokens (router GEMM + top-k softmax kernel);
2. order the T_local*k (token, expert) slots by owning rank; exchange per-rank counts
   (all-to-all of ``[ep]`` int64), then the token rows and their expert ids;
3. run the received rows through this rank's experts (align / grouped GEMM kernels with k=1);
4. all-to-all the results back and combine them with the routing weights.

With TP attention the tokens are already replicated on every rank, and
:class:`~polykey_service_amd.models.mixtral.MixtralMoE` instead computes local experts for all
tokens and all-reduces (one collective instead of two all-to-alls + an all-gather).
"""
from __future__ import annotations

import torch
import torch.nn.functional as F

from ..ops import moe as moe_ops
from . import comm
from .state import get_state


def moe_all_to_all(x: torch.Tensor, router_w: torch.Tensor, w13: torch.Tensor, w2: torch.Tensor, k: int) -> torch.Tensor:
    """x: this rank's tokens [T_local, H]; w13/w2: this rank's experts.  Returns [T_local, H]."""
    st = get_state()
    ep, r = st.tp_size, st.tp_rank
    E = router_w.shape[0]
    per = E // ep
    T = x.shape[0]
    logits = F.linear(x, router_w)
    ids, wts = moe_ops.topk_softmax(logits, k)
    flat = ids.reshape(-1).long()
    dest = flat // per
    order = torch.sort(dest, stable=True).indices
    send_counts = torch.bincount(dest, minlength=ep).to(torch.int64)
    recv_counts = comm.tp_all_to_all_counts(send_counts.to(x.device)).cpu()
    sc, rc = send_counts.tolist(), recv_counts.tolist()
    send_x = x.index_select(0, order // k)
    send_e = (flat[order] - dest[order] * per).to(torch.int32).view(-1, 1)
    recv_x = comm.tp_all_to_all(send_x, rc, sc)
    recv_e = comm.tp_all_to_all(send_e.to(x.device), rc, sc).view(-1, 1)
    n = recv_x.shape[0]
    if n > 0:
        ones = torch.ones((n, 1), dtype=torch.float32, device=x.device)
        offsets, sorted_, inv = moe_ops.align(recv_e, per, 0, per)
        xs = moe_ops.permute(recv_x, sorted_, offsets, 1)
        h = moe_ops.grouped_gemm(xs, w13, offsets, n, silu=True)
        y = moe_ops.grouped_gemm(h, w2, offsets, n, silu=False)
        y = moe_ops.unpermute(y, inv, ones, n, 1)
    else:
        y = recv_x
    back = comm.tp_all_to_all(y, sc, rc)
    # combine: slot order[i] received back[i]
    contrib = torch.zeros((T * k, x.shape[1]), dtype=torch.float32, device=x.device)
    contrib[order] = back.float()
    contrib = contrib.view(T, k, -1) * wts.view(T, k, 1).float()
    return contrib.sum(1).to(x.dtype)
