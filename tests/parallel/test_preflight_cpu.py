"""Multi-GPU preflight (parallel/preflight.py) on the CPU with 2 gloo ranks: the device-collective
paths are stood in for by correct gloo implementations with the same interfaces (the RCCL
communicator, the IPC custom all-reduce), one of them made faulty on ONE rank.  The check must
fail on that rank, the group must agree, the path must be disabled on BOTH ranks (no rank left
waiting in a collective its peer abandoned), the healthy path must stay, and the JSON log line
must name the fallback."""
import json
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


class GlooComm:
    """RcclComm's interface over the gloo group (correct)."""

    def __init__(self, group, world):
        self.g, self.nranks = group, world

    def all_reduce(self, x, op="sum", out=None):
        out = x if out is None else out.copy_(x)
        dist.all_reduce(out, group=self.g)
        return out

    def all_gather(self, x, out=None):
        parts = [torch.empty_like(x) for _ in range(self.nranks)]
        dist.all_gather(parts, x.contiguous(), group=self.g)
        return torch.cat(parts)

    def reduce_scatter(self, x, op="sum", out=None):
        y = x.clone()
        dist.all_reduce(y, group=self.g)
        return y.view(self.nranks, -1)[dist.get_rank(self.g)].clone()

    def all_to_allv(self, x, out_splits, in_splits):  # gloo has no all_to_all: exchange the row lists
        allp = [None] * self.nranks
        dist.all_gather_object(allp, list(x.split(in_splits)), group=self.g)
        me = dist.get_rank(self.g)
        return torch.cat([allp[j][me] for j in range(self.nranks)])


class BadGather(GlooComm):
    def all_gather(self, x, out=None):
        return super().all_gather(x) + 1  # a broken transport: every element off by one


class FakeCar:
    """custom_ar's all-gather / fused-collective interface over gloo (correct)."""

    def __init__(self, group, world):
        self.g, self.world, self.closed = group, world, False

    def supports_gather(self, x):
        return True

    def all_gather_last(self, x):
        parts = [torch.empty_like(x) for _ in range(self.world)]
        dist.all_gather(parts, x.contiguous(), group=self.g)
        return torch.cat(parts, -1)

    def supports_reduce_residual(self, M, N):
        return N % 1024 == 0

    def reduce_residual(self, pending, residual, parts):
        s = pending.float().clone()
        dist.all_reduce(s, group=self.g)
        residual.copy_((residual.float() + s).to(residual.dtype))
        M, N = residual.shape
        pv = parts.view(-1)[: (N // 1024) * M].view(N // 1024, M)
        pv.copy_(residual.float().view(M, N // 1024, 1024).pow(2).sum(-1).t())
        return pv

    def close(self):
        self.closed = True


def _worker(rank, world, port, out, faulty_rank):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank), POLYKEY_PREFLIGHT="0")
    from polykey_service_amd.parallel import preflight
    from polykey_service_amd.parallel.state import destroy_parallel, init_parallel
    st = init_parallel(tp=world, device="cpu", backend="gloo")
    st.rccl_tp = (BadGather if rank == faulty_rank else GlooComm)(st.tp_cpu_group, world)
    car = st.custom_ar = FakeCar(st.tp_cpu_group, world)
    lines = []
    rep = preflight.run(st, emit=lines.append)
    torch.save({"report": rep, "lines": lines, "rccl": st.rccl_tp is not None, "car": st.custom_ar is not None,
                "car_closed": car.closed}, f"{out}.{rank}")
    st.rccl_tp = st.custom_ar = None
    destroy_parallel()


@pytest.mark.parametrize("faulty_rank", [-1, 1])
def test_preflight_disables_a_faulty_collective_on_every_rank(tmp_path, faulty_rank):
    out = str(tmp_path / "pf")
    mp.start_processes(_worker, args=(2, _port(), out, faulty_rank), nprocs=2, join=True, start_method="spawn")
    res = [torch.load(f"{out}.{r}", weights_only=True) for r in range(2)]
    for r, d in enumerate(res):
        rep = d["report"]
        assert rep["checks"]["custom_ar"]["ok"] and d["car"] and not d["car_closed"], rep
        assert set(rep["checks"]["custom_ar"]) >= {"all_gather_1shot", "reduce_residual"}
        rc = rep["checks"]["rccl_tp"]
        assert rc.get("all_reduce") and rc.get("reduce_scatter") and rc.get("all_to_allv"), rc
        if faulty_rank < 0:
            assert rc["ok"] and rc["group_ok"] and d["rccl"] and rep["disabled"] == []
        else:
            assert rc["ok"] == (r != faulty_rank) and rc["all_gather"] == (r != faulty_rank)
            assert not rc["group_ok"] and not d["rccl"] and rep["disabled"] == ["rccl_tp"]  # on BOTH ranks
    # one JSON line from rank 0 always, and from the rank that saw the failure
    assert len(res[0]["lines"]) == 1 and json.loads(res[0]["lines"][0])["event"] == "multi_gpu_preflight"
    if faulty_rank >= 0:
        line = json.loads(res[faulty_rank]["lines"][0])
        assert line["disabled"] == ["rccl_tp"] and line["checks"]["rccl_tp"]["all_gather"] is False
    else:
        assert res[1]["lines"] == []
