"""Process-group bootstrap: one process per GPU, ``torch.distributed`` over RCCL ("nccl"
on ROCm) between GPUs of one node, gloo for CPU tests and for the CPU-side control plane.

Layout of a job with ``world`` ranks and tensor-parallel degree ``tp``:
``dp = world // tp`` independent replicas (request-level data parallel, SURVEY.md §2.3 "DP"),
each a TP group of consecutive ranks (``[r*tp, (r+1)*tp)``) so a TP group stays inside one
xGMI-connected node.  Expert parallelism (SURVEY.md §2.3 "EP") comes in two layouts:

* ``ep == tp``: EP inside the TP group (Mixtral EP=8 with attention TP=8): tokens are
  replicated by the TP attention, each rank computes its experts for all of them and the
  combine is the TP all-reduce;
* ``tp == 1, ep == world`` (*DP attention + EP*): every rank is its own attention / scheduling
  replica with its own requests, and the MoE layers exchange token rows with an expert
  all-to-all over the EP group (``parallel/ep.py``).  Ranks step in lockstep (LLMEngine).
"""
from __future__ import annotations

import dataclasses
import datetime
import logging
import os
from typing import List, Optional

import torch
import torch.distributed as dist

log = logging.getLogger(__name__)


@dataclasses.dataclass
class ParallelState:
    world_size: int = 1
    rank: int = 0
    local_rank: int = 0
    tp_size: int = 1
    tp_rank: int = 0
    tp_leader: int = 0                     # global rank of this TP group's first rank (its leader)
    dp_size: int = 1
    dp_rank: int = 0
    ep_size: int = 1
    ep_rank: int = 0
    ep_group: Optional[object] = None      # expert all-to-all (the TP group, or WORLD with DP attention)
    ep_cpu_group: Optional[object] = None  # gloo: DP-attention lockstep votes
    tp_group: Optional[object] = None      # device collectives (RCCL / gloo on CPU)
    tp_cpu_group: Optional[object] = None  # gloo: control-plane broadcast of step metadata
    custom_ar: Optional[object] = None     # one-shot xGMI all-reduce (parallel/custom_ar.py)
    rccl_tp: Optional[object] = None       # direct RCCL communicator of the TP group (parallel/rccl.py)
    rccl_ep: Optional[object] = None       # ... of the EP group (the TP one when EP runs inside TP)
    ep_a2a: Optional[object] = None        # IPC expert all-to-all (parallel/ep_ipc.py; DP attention + EP)
    ep_board: Optional[object] = None      # shared-memory lockstep vote (csrc/runtime/vote_board.cpp)
    ep_a2a_prefill: Optional[object] = None  # IPC expert all-to-all sized for prefill steps (eager)
    ep_step_rows: int = 1 << 30            # largest token count of the current lockstep step (vote)
    backend: str = "none"
    device: torch.device = dataclasses.field(default_factory=lambda: torch.device("cpu"))
    # several local ranks on one GPU (rehearsals): kernels whose workgroups wait on each other
    # in-launch (gemm.mlp_fused) assume the whole grid is resident, which another process's
    # waiting grid can prevent -- they are not used then
    shared_device: bool = False
    # ranks of this job on this rank's physical GPU (counted by device identity, not inferred
    # from LOCAL_WORLD_SIZE vs the visible-device count: a rank per GPU that sees only its own
    # device through HIP_VISIBLE_DEVICES is not sharing)
    ranks_per_device: int = 1
    world_cpu_group: Optional[object] = None  # gloo over every rank (start-up exchanges)

    @property
    def is_tp_leader(self) -> bool:
        return self.tp_rank == 0

    @property
    def distributed(self) -> bool:
        return self.world_size > 1

    @property
    def dp_attention(self) -> bool:
        """Attention replicated per rank (tp = 1) with experts spread over ep > 1 ranks."""
        return self.ep_size > 1 and self.tp_size == 1


_STATE = ParallelState()


def get_state() -> ParallelState:
    return _STATE


def set_state(st: ParallelState) -> None:
    global _STATE
    _STATE = st


def pick_backend(dev_type: str, n_dev: int, local_world: int, override: Optional[str] = None) -> str:
    """RCCL ("nccl") for one rank per GPU; gloo on CPU and when a node runs more local ranks
    than it has GPUs (RCCL refuses two ranks on one device); ``override`` wins."""
    if override:
        return override
    return "nccl" if dev_type == "cuda" and local_world <= max(n_dev, 1) else "gloo"


def init_parallel(tp: int = 1, ep: int = 1, device: Optional[str] = None, backend: Optional[str] = None,
                  timeout_s: float = 600.0, tp_groups: Optional[List[List[int]]] = None) -> ParallelState:
    """Initialise from torchrun-style env (RANK / WORLD_SIZE / LOCAL_RANK / MASTER_*).
    Without WORLD_SIZE (or WORLD_SIZE=1) returns a single-process state and creates no group.
    ``tp_groups``: explicit TP groups of consecutive ranks, possibly of different sizes (several
    models behind one front end, adapters/local_llm.py plan_model_groups); ``tp`` is then this
    rank's group size and ``dp`` counts the groups."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", str(rank)))
    if device is None:
        device = "cuda" if torch.cuda.is_available() else "cpu"
    # more local ranks than GPUs (rehearsing a multi-rank launch on a one-GPU box) share devices
    n_dev = torch.cuda.device_count() if device == "cuda" else 0
    dev = torch.device(f"cuda:{local % max(n_dev, 1)}") if device == "cuda" else torch.device(device)
    if dev.type == "cuda":
        torch.cuda.set_device(dev)
    if tp_groups is not None:
        if sorted(r for g in tp_groups for r in g) != list(range(world)) or any(
                g != list(range(g[0], g[0] + len(g))) for g in tp_groups):
            raise ValueError(f"tp_groups {tp_groups} must split ranks 0..{world - 1} into consecutive runs")
        if ep != 1:
            raise ValueError("explicit TP groups serve dense / TP-sharded models only (ep = 1)")
        mine = next(g for g in tp_groups if rank in g)
        tp = len(mine)
    else:
        if world % tp:
            raise ValueError(f"world size {world} not divisible by tp={tp}")
        tp_groups = [list(range(r * tp, (r + 1) * tp)) for r in range(world // tp)]
        mine = tp_groups[rank // tp]
    dp_attn = tp == 1 and ep > 1
    if dp_attn and ep != world:
        raise ValueError(f"DP attention + EP needs ep == world size ({world}), got ep={ep}")
    if not dp_attn and ep not in (1, tp):
        raise ValueError("expert parallelism must be 1, equal to tp (EP inside the TP group), or the world size "
                         "with tp=1 (DP attention + expert all-to-all)")
    st = ParallelState(world_size=world, rank=rank, local_rank=local, tp_size=tp, tp_rank=rank - mine[0],
                       tp_leader=mine[0],
                       dp_size=len(tp_groups), dp_rank=tp_groups.index(mine), ep_size=ep,
                       ep_rank=rank if dp_attn else ((rank % tp) if ep > 1 else 0), device=dev)
    if world > 1:
        # POLYKEY_DIST_BACKEND overrides (gloo: several ranks on one GPU, which RCCL refuses)
        be = pick_backend(dev.type, n_dev, int(os.environ.get("LOCAL_WORLD_SIZE", "1")),
                          backend or os.environ.get("POLYKEY_DIST_BACKEND"))
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        # a hung or failed RCCL collective aborts the communicator and raises in this process
        # (timeout_s), which takes the engine down → health NOT_SERVING → supervisor restart
        os.environ.setdefault("TORCH_NCCL_ASYNC_ERROR_HANDLING", "1")
        if not dist.is_initialized():
            kw = dict(backend=be, timeout=datetime.timedelta(seconds=timeout_s))
            if be == "nccl":
                kw["device_id"] = dev
            dist.init_process_group(**kw)
        st.backend = be
        st.world_cpu_group = dist.group.WORLD if be == "gloo" else dist.new_group(list(range(world)), backend="gloo")
        st.ranks_per_device = _ranks_on_my_device(st)
        st.shared_device = dev.type == "cuda" and st.ranks_per_device > 1
        for ranks in tp_groups:  # every rank creates every group, in the same order (collective)
            g = dist.new_group(ranks) if len(ranks) < world else dist.group.WORLD
            gc = dist.new_group(ranks, backend="gloo") if be != "gloo" else g
            if rank in ranks:
                st.tp_group, st.tp_cpu_group = g, gc
        if dp_attn:
            st.ep_group = dist.group.WORLD
            # a dedicated gloo group: the engine thread's lockstep votes must never interleave
            # with another thread's collectives on WORLD
            st.ep_cpu_group = dist.new_group(list(range(world)), backend="gloo")
            st.ep_board = _vote_board(st)
        elif ep > 1:
            st.ep_group, st.ep_cpu_group = st.tp_group, st.tp_cpu_group
        if be == "nccl" or (os.environ.get("POLYKEY_CUSTOM_AR") == "force" and dev.type == "cuda"):
            from .custom_ar import maybe_create
            st.custom_ar = maybe_create(st)
        if be == "nccl" and os.environ.get("POLYKEY_RCCL_DIRECT", "1") == "1":
            _create_rccl(st)
        # every device collective path checked once on a few KB before the first step; a failed
        # one is disabled on all ranks (parallel/preflight.py).  POLYKEY_PREFLIGHT=0 skips it.
        if os.environ.get("POLYKEY_PREFLIGHT", "1") != "0" and (st.rccl_tp is not None or st.rccl_ep is not None
                                                                 or st.custom_ar is not None):
            from . import preflight
            preflight.run(st)
    set_state(st)
    return st


def device_identity(dev: torch.device) -> str:
    """Host + PCI address + UUID of a GPU (what two processes compare to tell whether they share
    one physical device); the host alone for CPU ranks (never 'sharing')."""
    import socket
    host = socket.gethostname()
    if dev.type != "cuda":
        return f"{host}/cpu/{os.getpid()}"
    p = torch.cuda.get_device_properties(dev)
    return f"{host}/{p.pci_domain_id:04x}:{p.pci_bus_id:02x}:{p.pci_device_id:02x}/{p.uuid}"


def _ranks_on_my_device(st: ParallelState) -> int:
    ids = [None] * st.world_size
    dist.all_gather_object(ids, device_identity(st.device), group=st.world_cpu_group)
    mine = ids[st.rank]
    return sum(1 for i in ids if i == mine)


def _vote_board(st: ParallelState):
    """Shared-memory lockstep vote for the DP-attention + EP ranks of ONE node (the gloo vote
    stays for multi-node groups)."""
    if int(os.environ.get("LOCAL_WORLD_SIZE", str(st.world_size))) != st.world_size:
        return None
    import uuid

    from .._native.loader import load_extension
    board, err = None, None
    name = [None]
    try:
        rt = load_extension("_pk_runtime")
        if st.rank == 0:  # created before its name is published: attaching can never race it
            name[0] = f"/pk_vote_{os.getpid()}_{uuid.uuid4().hex[:8]}"
            board = rt.VoteBoard(name[0], True, st.world_size, 0)
    except Exception as e:  # noqa: BLE001
        err = e
    dist.broadcast_object_list(name, src=0, group=st.ep_cpu_group)
    if st.rank != 0 and name[0] is not None:
        try:
            board = rt.VoteBoard(name[0], False, st.world_size, st.rank)
        except Exception as e:  # noqa: BLE001
            err = e
    ok = [None] * st.world_size
    dist.all_gather_object(ok, board is not None, group=st.ep_cpu_group)  # all ranks or none
    if not all(ok):
        log.warning("shared-memory vote board unavailable (%s); lockstep votes over gloo", err)
        return None
    if st.rank == 0:
        board.unlink()  # every rank attached: nothing left in /dev/shm if the group is killed
    return board


def _create_rccl(st: ParallelState) -> None:
    """Direct RCCL communicators for the TP and EP groups (collective over each group; the
    unique ids travel over the gloo groups).  Any failure leaves torch.distributed in charge."""
    from . import rccl
    try:
        if st.tp_size > 1:
            st.rccl_tp = rccl.RcclComm.create(st.tp_group, st.device, cpu_group=st.tp_cpu_group)
        if st.ep_size > 1:
            st.rccl_ep = (st.rccl_tp if st.ep_group is st.tp_group
                          else rccl.RcclComm.create(st.ep_group, st.device, cpu_group=st.ep_cpu_group))
    except (rccl.RcclError, OSError) as e:  # pragma: no cover - needs several GPUs
        log.warning("direct RCCL communicators unavailable (%s); collectives stay on torch.distributed", e)
        st.rccl_tp = st.rccl_ep = None


def destroy_parallel() -> None:
    st = get_state()
    if st.custom_ar is not None:
        st.custom_ar.close()
    for a2a in (st.ep_a2a, st.ep_a2a_prefill):
        if a2a is not None:
            a2a.close()
    for c in {id(c): c for c in (st.rccl_tp, st.rccl_ep) if c is not None}.values():
        c.close()
    if dist.is_initialized():
        dist.destroy_process_group()
    set_state(ParallelState())
