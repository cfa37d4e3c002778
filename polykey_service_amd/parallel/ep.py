"""Expert parallelism with all-to-all dispatch / combine (DP attention + EP).

Each EP rank runs attention for its *own* requests (``ParallelState.dp_attention``: tp = 1,
ep = world) and owns experts ``[r*E/ep, (r+1)*E/ep)``.  Per MoE layer (SURVEY.md §2.3
"Mixtral EP all-to-all"; BASELINE.json config 5):

1. route the local tokens (router GEMM + the top-k softmax kernel, or the routing the fused
   residual-add + RMSNorm kernel already produced);
2. order the ``T_local * k`` (token, slot) pairs by owning rank with the expert-align
   counting sort keyed by destination rank, gather the rows into that order (the MoE permute
   kernel) -- the send buffer is contiguous per destination;
3. exchange the rows and their expert ids: on one node through fixed-capacity IPC regions with
   device-side counts (:mod:`.ep_ipc`, graph-capturable), otherwise per-destination counts
   (one int64 all-to-all and a host read-back) and two variable-size all-to-alls over RCCL;
4. the received rows run through this rank's experts (align / grouped GEMM with the SiLU
   epilogue / grouped GEMM, k = 1) and are put back into arrival order;
5. the results travel back with the inverse all-to-all, landing in the same per-destination
   order the rows left in, so the combine is the ordinary weighted un-permute of the MoE
   kernels -- deferred into the next residual add + RMSNorm kernel when the caller allows.

A rank with no tokens this step still takes part (it sends nothing and serves the others'
rows): :meth:`~polykey_service_amd.models.mixtral.MixtralForCausalLM.idle_forward`.

With attention TP (``ep == tp``) the tokens are already replicated on every rank and
:class:`~polykey_service_amd.models.mixtral.MixtralMoE` computes local experts for all of them
and all-reduces instead (one collective instead of two all-to-alls).
"""
from __future__ import annotations

from typing import Optional, Tuple

import torch
import torch.nn.functional as F

from ..ops import moe as moe_ops
from . import comm
from .state import get_state


def _local_experts(recv_x: torch.Tensor, recv_e: torch.Tensor, w13: torch.Tensor, w2: torch.Tensor,
                   w13_p: Optional[torch.Tensor], w2_p: Optional[torch.Tensor], rows: Optional[int] = None,
                   bound: Optional[int] = None) -> torch.Tensor:
    """Rows received from every rank × their local expert → outputs in arrival order (rows whose
    expert id is not local -- the IPC regions' -1 padding -- come out as zeros).  ``bound``: an
    upper bound of any one expert's rows (the grouped GEMM's tile choice) when the counts live on
    the device."""
    n = recv_x.shape[0] if rows is None else rows
    if n == 0:
        return recv_x
    per = w13.shape[0]
    offsets, sorted_, inv = moe_ops.align(recv_e, per, 0, per)
    xs = moe_ops.permute(recv_x, sorted_, offsets, 1)
    mr = n if bound is None else bound
    h = moe_ops.grouped_gemm(xs, w13, offsets, mr, silu=True, packed=w13_p)
    y = moe_ops.grouped_gemm(h, w2, offsets, mr, silu=False, packed=w2_p)
    ones = torch.ones((n, 1), dtype=torch.float32, device=recv_x.device)
    return moe_ops.unpermute(y, inv, ones, n, 1)


def ep_moe(x: torch.Tensor, router_w: torch.Tensor, w13: torch.Tensor, w2: torch.Tensor, k: int,
           routing: Optional[Tuple[torch.Tensor, torch.Tensor]] = None, w13_p: Optional[torch.Tensor] = None,
           w2_p: Optional[torch.Tensor] = None, defer_combine: bool = False):
    """x: this rank's tokens [T_local, H] (T_local may be 0); w13 / w2: this rank's experts.
    Returns [T_local, H], or a :class:`~polykey_service_amd.ops.moe.PendingCombine`.

    The step's path is uniform over the EP group (every rank must issue the same collectives):
    the IPC all-to-all when the step's largest token count fits its capacity (``st.ep_step_rows``
    from the lockstep vote), else the RCCL / gloo all-to-all with split lists on the host.  On
    one node the IPC regions cover every step -- the decode set sized for ``max_num_seqs`` x k
    rows per peer, the prefill set for the whole ``max_num_batched_tokens`` x k token budget
    (llm_engine.py; ~1.2 GB of receive + return regions per rank for Mixtral at 8192 tokens,
    EP = 8) -- so the per-layer count read-back below runs only where those regions do not
    exist: across nodes, on CPU / gloo, or after the multi-GPU preflight disabled the IPC path."""
    st = get_state()
    for a2a in (st.ep_a2a, st.ep_a2a_prefill):  # decode-sized regions first, then prefill-sized
        if a2a is not None and x.is_cuda and a2a.fits(st.ep_step_rows * k):
            return _ep_moe_ipc(a2a, x, router_w, w13, w2, k, routing, w13_p, w2_p, defer_combine)
    ep = st.ep_size
    E = router_w.shape[0]
    per = E // ep
    T, H = x.shape
    dev = x.device
    if T > 0:
        ids, wts = routing if routing is not None else moe_ops.topk_softmax(F.linear(x, router_w), k)
        dest = torch.div(ids, per, rounding_mode="floor").to(torch.int32)
        offsets, sorted_, inv = moe_ops.align(dest, ep, 0, ep)  # every slot is "local" in rank space
        send_x = moe_ops.permute(x, sorted_, offsets, k)
        sl = sorted_.long()
        send_e = (ids.reshape(-1).long()[sl] - dest.reshape(-1).long()[sl] * per).to(torch.int32).view(-1, 1)
        send_counts = (offsets[1:] - offsets[:-1]).to(torch.int64)
    else:
        ids = torch.zeros((0, k), dtype=torch.int32, device=dev)
        wts = torch.zeros((0, k), dtype=torch.float32, device=dev)
        inv = torch.zeros((0,), dtype=torch.int32, device=dev)
        send_x = x
        send_e = torch.zeros((0, 1), dtype=torch.int32, device=dev)
        send_counts = torch.zeros(ep, dtype=torch.int64, device=dev)
    recv_counts = comm.ep_all_to_all_counts(send_counts.to(dev))
    counts = torch.stack([send_counts.to(dev), recv_counts]).cpu()  # one read-back for both
    sc, rc = counts[0].tolist(), counts[1].tolist()
    recv_x = comm.ep_all_to_all(send_x, rc, sc)
    recv_e = comm.ep_all_to_all(send_e, rc, sc).view(-1, 1)
    y = _local_experts(recv_x, recv_e, w13, w2, w13_p, w2_p)
    back = comm.ep_all_to_all(y, sc, rc)  # [T*k, H] in the send (destination-sorted) order
    pending = moe_ops.PendingCombine(back, inv, wts, T, k)
    if defer_combine and T > 0:
        return pending
    return pending.combine() if T > 0 else x.new_zeros((0, H))


def _ep_moe_ipc(a2a, x, router_w, w13, w2, k, routing, w13_p, w2_p, defer_combine):
    """ep_moe over the IPC regions: device-side counts and offsets only (graph-capturable)."""
    st = get_state()
    ep = st.ep_size
    E = router_w.shape[0]
    per = E // ep
    T, H = x.shape
    dev = x.device
    if T > 0:
        ids, wts = routing if routing is not None else moe_ops.topk_softmax(F.linear(x, router_w), k)
        dest = torch.div(ids, per, rounding_mode="floor").to(torch.int32)
        offsets, sorted_, inv = moe_ops.align(dest, ep, 0, ep)  # destination-sorted (token, slot) rows
        send_x = moe_ops.permute(x, sorted_, offsets, k)
        sl = sorted_.long()
        send_e = (ids.reshape(-1).long()[sl] - dest.reshape(-1).long()[sl] * per).to(torch.int32)
    else:
        wts = torch.zeros((0, k), dtype=torch.float32, device=dev)
        inv = torch.zeros((0,), dtype=torch.int32, device=dev)
        send_x = x
        send_e = torch.zeros((0,), dtype=torch.int32, device=dev)
        offsets = torch.zeros(ep + 1, dtype=torch.int32, device=dev)
    a2a.dispatch(send_x.contiguous(), send_e, offsets)
    # every rank's rows are in this rank's receive regions (padding ids -1: no local expert)
    n = ep * a2a.C
    # any one local expert gets at most one row per token of every sender, and no sender has more
    # than the step's largest token count (the lockstep vote's max; a captured graph's bucket, and
    # every rank replays the bucket of the vote's max: ModelRunner.launch)
    bound = ep * min(st.ep_step_rows, a2a.C)
    y = _local_experts(a2a.recv_x, a2a.recv_e.view(-1, 1), w13, w2, w13_p, w2_p, rows=n, bound=bound)
    back = a2a.return_(y.contiguous())[: T * k]  # this rank's rows, in the order they were sent
    pending = moe_ops.PendingCombine(back, inv, wts, T, k)
    if defer_combine and T > 0:
        return pending
    return pending.combine() if T > 0 else x.new_zeros((0, H))


def moe_all_to_all(x: torch.Tensor, router_w: torch.Tensor, w13: torch.Tensor, w2: torch.Tensor, k: int) -> torch.Tensor:
    """Combined expert output for this rank's tokens (see :func:`ep_moe`)."""
    return ep_moe(x, router_w, w13, w2, k)
