"""Debug probe: IPC all-gather / fused reduce at W ranks sharing one GPU (prints mismatches)."""
import os
import socket
import sys

import torch
import torch.distributed as dist
import torch.multiprocessing as mp

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.cuda.set_device(0)
    from polykey_service_amd.parallel.custom_ar import CustomAllReduce
    dev = torch.device("cuda:0")
    car = CustomAllReduce(dist.group.WORLD, rank, world, dev, max_bytes=1 << 22, blocks=4, timeout_s=20.0)
    ok = car.self_test()
    msgs = [f"self_test={ok}"]
    from polykey_service_amd.ops.gemm import Partial
    seq = []
    for M in (1, 3, 64):
        if os.environ.get("PROBE_FUSED") == "1":
            N = 1024
            res = torch.zeros(M, N, dtype=torch.bfloat16, device=dev)
            parts = torch.zeros(64 * 8, dtype=torch.float32, device=dev)
            slabs = torch.full((2 * M * N,), float(rank), dtype=torch.float32, device=dev)
            car.fused_blocks = 32
            car.reduce_residual(Partial(slabs, 2, M, N), res, parts)
            torch.cuda.synchronize()
            want = float(sum(2 * r for r in range(world)))
            msgs.append(f"fused M={M} res_ok={bool((res.float() == want).all())} v={float(res[0,0])} err={car.error()}")
        for cols in (256, 1024):
            lg = torch.full((M, cols), float(rank), dtype=torch.bfloat16, device=dev)
            got = car.all_gather_last(lg)
            torch.cuda.synchronize()
            g = got.cpu().view(M, world, cols).float()
            want = torch.arange(world, dtype=torch.float32).view(1, world, 1).expand(M, world, cols)
            bad = (g != want)
            if bad.any():
                idx = bad.nonzero()[:5].tolist()
                msgs.append(f"M={M} cols={cols} bad={int(bad.sum())}/{bad.numel()} first={idx} "
                            f"vals={[float(g[i][j][k]) for i, j, k in idx]}")
            else:
                msgs.append(f"M={M} cols={cols} ok")
    msgs.append(f"err={car.error()}")
    dist.barrier()
    car.close()
    q.put((rank, msgs))


if __name__ == "__main__":
    for world in (2, 8):
        s = socket.socket()
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
        s.close()
        ctx = mp.get_context("spawn")
        q = ctx.Queue()
        ps = [ctx.Process(target=worker, args=(r, world, port, q)) for r in range(world)]
        for p in ps:
            p.start()
        res = dict(q.get(timeout=120) for _ in ps)
        for p in ps:
            p.join(30)
        print(f"world={world}", flush=True)
        for r in sorted(res):
            print(r, res[r], flush=True)
