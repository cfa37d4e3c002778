"""Wiring of the direct RCCL communicators into parallel/comm.py, checked on the CPU with a
recording stand-in (RCCL itself needs GPUs: tests/parallel/test_rccl_gpu.py).  Every TP / SP /
EP device collective must reach the communicator with the right buffers, splits and in-place
semantics -- the paths only a multi-GPU node would otherwise exercise."""
import pytest
import torch

from polykey_service_amd.parallel import comm
from polykey_service_amd.parallel.state import ParallelState, get_state, set_state


class FakeComm:
    """Two-rank communicator seen from rank 0 whose peer contributes ones / mirrors rows."""

    def __init__(self, n=2):
        self.nranks, self.calls = n, []

    def all_reduce(self, x, op="sum", out=None):
        self.calls.append(("all_reduce", tuple(x.shape)))
        out = x if out is None else out
        out.copy_(x + 1)
        return out

    def all_gather(self, x, out=None):
        self.calls.append(("all_gather", tuple(x.shape)))
        res = torch.cat([x, x + 100])
        if out is None:
            return res
        out.view(-1).copy_(res.view(-1))
        return out

    def reduce_scatter(self, x, op="sum", out=None):
        self.calls.append(("reduce_scatter", tuple(x.shape)))
        res = x[: x.shape[0] // 2] * 2
        if out is None:
            return res
        out.copy_(res)
        return out

    def broadcast(self, x, root=0):
        self.calls.append(("broadcast", root))
        return x

    def all_to_allv(self, x, out_splits, in_splits):
        self.calls.append(("all_to_allv", list(out_splits), list(in_splits)))
        assert sum(in_splits) == x.shape[0]
        # the peer sends back exactly what it was sent (symmetric exchange)
        return x.clone()[: sum(out_splits)]


@pytest.fixture()
def fake_state(monkeypatch):
    old = get_state()
    fc = FakeComm()
    st = ParallelState(world_size=2, tp_size=2, ep_size=2, rccl_tp=fc, rccl_ep=fc)
    set_state(st)
    monkeypatch.setattr(comm, "_direct", lambda c, x: c)  # route CPU tensors too
    yield fc
    set_state(old)


def test_tp_collectives_use_the_direct_communicator(fake_state):
    fc = fake_state
    x = torch.zeros(4, 8)
    assert comm.tp_all_reduce(x) is x and torch.all(x == 1)  # in place
    g = comm.tp_all_gather_last(torch.arange(6.0).view(2, 3))
    assert g.shape == (2, 6) and torch.equal(g[:, 3:], g[:, :3] + 100)  # rank-major along the last dim
    out = comm.tp_all_to_all(torch.arange(10.0).view(5, 2), [2, 3], [1, 4])
    assert out.shape == (5, 2)
    cnt = comm.tp_all_to_all_counts(torch.tensor([3, 4]))
    assert torch.equal(cnt, torch.tensor([3, 4]))
    b = torch.ones(3)
    assert comm.tp_broadcast_tensor(b) is b
    assert [c[0] for c in fc.calls] == ["all_reduce", "all_gather", "all_to_allv", "all_to_allv", "broadcast"]
    assert fc.calls[2][1:] == ([2, 3], [1, 4]) and fc.calls[3][1:] == ([1, 1], [1, 1])


def test_sp_reduce_scatter_and_gather_use_the_direct_communicator(fake_state):
    fc = fake_state
    lay = comm.SPLayout(8, chunks=1)
    lay.tp, lay.rank = 2, 0
    y = torch.arange(16.0).view(8, 2)
    shard = comm.sp_reduce_scatter(y, lay)
    assert torch.equal(shard, y[:4] * 2)
    full = comm.sp_all_gather(shard, lay)
    assert full.shape == (8, 2)
    assert [c[0] for c in fc.calls] == ["reduce_scatter", "all_gather"]


def test_ep_all_to_all_uses_the_direct_communicator(fake_state, monkeypatch):
    fc = fake_state
    monkeypatch.setattr(comm.dist, "get_backend", lambda g=None: "nccl")
    x = torch.arange(12.0).view(6, 2)
    out = comm.ep_all_to_all(x, [6, 0], [2, 4])
    assert torch.equal(out, x)
    cnt = comm.ep_all_to_all_counts(torch.tensor([2, 4]))
    assert torch.equal(cnt, torch.tensor([2, 4]))
    assert fc.calls == [("all_to_allv", [6, 0], [2, 4]), ("all_to_allv", [1, 1], [1, 1])]
