"""One-shot / two-shot xGMI all-reduce (csrc/comm/custom_allreduce.hip) with 2 and 8 ranks.

On a one-GPU box all ranks share cuda:0: IPC handles, peer flags, parity slots and graph
replay are exercised exactly as across GPUs (the loads just do not cross xGMI); 8 ranks run
the W=8 instantiation that 70B TP=8 uses.  Small grids keep every rank's kernels co-resident;
every wait is bounded by a wall-clock timeout that sets the sticky error word (no hang).
The last phase provokes that timeout on purpose: one rank skips a call."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu


def _port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        dist.init_process_group("gloo", rank=rank, world_size=world)
        torch.cuda.set_device(0)
        from polykey_service_amd.parallel.custom_ar import CustomAllReduce
        dev = torch.device("cuda:0")
        car = CustomAllReduce(dist.group.WORLD, rank, world, dev, max_bytes=1 << 22, blocks=4, timeout_s=20.0)
        assert car.self_test(), "self test"
        g = torch.Generator().manual_seed(100 + rank)
        for n in (8, 1000 * 8, 64 * 4096, 64 * 8192):
            x = torch.randn(n, generator=g).to(torch.bfloat16)
            xs = [torch.empty_like(x) for _ in range(world)]
            dist.all_gather(xs, x)
            exp = torch.stack([t.float() for t in xs]).sum(0)
            for algo in (0, 1, 2):  # by size, one-shot, two-shot (reduce-scatter + all-gather)
                y = car.all_reduce(x.to(dev), algo=algo).cpu().float()
                torch.testing.assert_close(y, exp.to(torch.bfloat16).float(), atol=1e-2, rtol=1e-2)
            xi = x.to(dev)
            car.all_reduce(xi, out=xi, algo=2)  # in place
            torch.testing.assert_close(xi.cpu().float(), exp.to(torch.bfloat16).float(), atol=1e-2, rtol=1e-2)
        # graph replay: the epoch lives in device memory, so replays stay in step
        xin = torch.zeros(4096, dtype=torch.bfloat16, device=dev)
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            car.all_reduce(xin)
        torch.cuda.current_stream().wait_stream(s)
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph):
            yg = car.all_reduce(xin)
        for it in range(3):
            xin.fill_(float(rank + it))
            dist.barrier()
            graph.replay()
            torch.cuda.synchronize()
            want = float(sum(r + it for r in range(world)))
            assert bool((yg.float() == want).all()), (it, yg[:4])
        assert car.error() == 0
        # a rank that skips a call: every rank that waits for it times out and fails loudly
        # (sticky error word, read without a GPU sync), and later calls return at once
        car.set_timeout(1.0)
        dist.barrier()
        if rank != world - 1:
            import time
            xs = torch.ones(4096, dtype=torch.bfloat16, device=dev)
            car.all_reduce(xs)
            torch.cuda.synchronize()
            assert car.error() == 1, "timeout not reported"
            t0 = time.monotonic()
            car.all_reduce(xs)
            torch.cuda.synchronize()
            assert time.monotonic() - t0 < 0.5, "a failed group must not wait again"
            from polykey_service_amd.parallel.custom_ar import CustomAllReduceError
            try:
                car.check()
                raise AssertionError("check() did not raise")
            except CustomAllReduceError:
                pass
        dist.barrier()
        car.close()
        dist.barrier()
        dist.destroy_process_group()
        q.put((rank, "ok"))
    except BaseException as e:  # noqa: BLE001
        q.put((rank, repr(e)))


@pytest.mark.parametrize("world", [2, 8])
def test_custom_allreduce_ranks_share_one_gpu(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=240) for _ in procs)
    for p in procs:
        p.join(timeout=60)
    assert res == {r: "ok" for r in range(world)}, res
