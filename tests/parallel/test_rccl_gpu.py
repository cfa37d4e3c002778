"""Direct RCCL communicators on one MI355X (a one-rank communicator: RCCL refuses two ranks on
one device, so the multi-rank paths run only on a multi-GPU node): every collective of the
binding returns the one-rank result on the caller's stream, works inside a captured HIP graph,
and the health poll reports no error."""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def comm():
    from polykey_service_amd.parallel import rccl
    c = rccl.RcclComm.single()
    yield c
    c.close()


def test_collectives_one_rank(comm):
    g = torch.Generator(device="cuda").manual_seed(0)
    x = torch.randn(4096, device="cuda", generator=g).to(torch.bfloat16)
    assert torch.equal(comm.all_reduce(x.clone()), x)
    y = x.clone()
    assert comm.all_reduce(y, out=y).data_ptr() == y.data_ptr() and torch.equal(y, x)
    m = torch.randn(64, 128, device="cuda", generator=g)
    assert torch.equal(comm.all_reduce(m, op="max"), m)
    assert torch.equal(comm.all_gather(m), m)
    assert torch.equal(comm.reduce_scatter(m), m)
    b = m.clone()
    assert torch.equal(comm.broadcast(b, root=0), m)
    rows = torch.randn(37, 256, device="cuda", generator=g).to(torch.bfloat16)
    assert torch.equal(comm.all_to_allv(rows, [37], [37]), rows)
    cnt = torch.tensor([5], dtype=torch.int64, device="cuda")
    assert torch.equal(comm.all_to_allv(cnt.view(-1, 1), [1], [1]).view(-1), cnt)
    comm.check()


def test_all_to_allv_empty_rows(comm):
    """An idle EP rank sends and receives [0, H]: zero counts everywhere must be a no-op."""
    empty = torch.zeros((0, 4096), dtype=torch.bfloat16, device="cuda")
    out = comm.all_to_allv(empty, [0], [0])
    torch.cuda.synchronize()
    assert out.shape == (0, 4096)
    comm.check()


def test_bad_arguments_raise(comm):
    x = torch.zeros(8, 8, device="cuda")
    with pytest.raises(ValueError):
        comm.all_to_allv(x, [8], [4])  # in_splits must cover the rows
    with pytest.raises(ValueError):
        comm.all_reduce(x.t())  # not contiguous
    with pytest.raises(TypeError):
        comm.all_reduce(torch.zeros(4, dtype=torch.bool, device="cuda"))


def test_all_reduce_in_a_hip_graph(comm):
    x = torch.ones(1 << 16, device="cuda", dtype=torch.bfloat16)
    out = torch.empty_like(x)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        comm.all_reduce(x, out=out)  # warm-up outside capture
    torch.cuda.current_stream().wait_stream(s)
    graph = torch.cuda.CUDAGraph()
    # captured like the engine captures its decode graphs: under inference mode (the CUDA
    # generator's graph-capture state is then an inference tensor for every later capture)
    with torch.inference_mode(), torch.cuda.graph(graph):
        comm.all_reduce(x, out=out)
    x.fill_(3.0)
    graph.replay()
    torch.cuda.synchronize()
    assert torch.all(out == 3.0)
    comm.check()
