"""One-shot / two-shot xGMI all-reduce (csrc/comm/custom_allreduce.hip) with 2, 4 and 8 ranks.

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
        _fused_phase(car, rank, world, dev)
        _serving_phase(car, rank, world, dev)
        # the fenced slot protocol (preflight's fallback): the same bits, and the
        # serving-shape check passes with it too; then back to the fence-free default
        car.set_fenced(True)
        assert car.fenced and not car.push_ok(64, 8192, 64)
        dist.barrier()
        _fused_phase(car, rank, world, dev)
        _serving_phase(car, rank, world, dev)
        car.set_fenced(False)
        dist.barrier()
        _overlap_phase(car, rank, world, dev)
        _carry_phase(car, rank, world, dev)
        _push_phase(car, rank, world, dev)
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
        import traceback
        q.put((rank, repr(e) + " " + traceback.format_exc()[-1500:]))


def _rr_reference(slabs_all, partials_all, res, S, nparts=None):
    """Sequential fp32 reference of pk_car_reduce_residual (same summation order); parts per
    N / nparts columns (1024: one-shot; 256: the two-shot form at 4+ ranks)."""
    world = len(partials_all)
    parts_bf = []
    for j in range(world):
        if S == 0:
            parts_bf.append(partials_all[j].float())
        else:
            a = torch.zeros_like(slabs_all[j][0])
            for s_ in range(S):
                a = a + slabs_all[j][s_]
            parts_bf.append(a.to(torch.bfloat16).float())
    acc = torch.zeros_like(parts_bf[0])
    for j in range(world):
        acc = acc + parts_bf[j]
    new = (acc.to(torch.bfloat16).float() + res.float()).to(torch.bfloat16)
    M, N = res.shape
    nparts = nparts or N // 1024
    sq = new.float().view(M, nparts, N // nparts).pow(2).sum(-1).t().contiguous()
    return new, sq


def _fused_phase(car, rank, world, dev):
    """Fused TP decode collective: slab reduce + peer sum + residual add + norm parts, eager and
    graph-replayed, interleaved with all-gathers and all-reduces of other grid sizes (one call
    epoch for every collective of the context)."""
    car.fused_blocks = 32  # every rank's grid resident at once on the shared GPU
    g = torch.Generator().manual_seed(7)  # same residual on every rank
    gr = torch.Generator().manual_seed(1000 + rank)
    # (4, 8192, 3) / (8, 4096, 4): one item per workgroup -- the two-shot form's slab prefetch ahead
    # of the epoch (S = 3 re-reads slab 2 past S, unsummed)
    for M, N, S in ((1, 1024, 2), (3, 4096, 0), (64, 8192, 4), (17, 2048, 1), (4, 8192, 3), (8, 4096, 4)):
        res = (torch.randn(M, N, generator=g) * 2).to(torch.bfloat16)
        slabs = torch.randn(max(S, 1), M, N, generator=gr) if S else None
        partial = torch.randn(M, N, generator=gr).to(torch.bfloat16) if S == 0 else None
        all_slabs = [torch.empty(max(S, 1), M, N) for _ in range(world)] if S else None
        all_part = [torch.empty(M, N, dtype=torch.bfloat16) for _ in range(world)]
        if S:
            dist.all_gather(all_slabs, slabs)
        else:
            dist.all_gather(all_part, partial)
        from polykey_service_amd.ops.gemm import Partial
        r_dev = res.to(dev)
        parts = torch.zeros((N // 256) * M, dtype=torch.float32, device=dev)
        pend = Partial(slabs.to(dev).reshape(-1), S, M, N) if S else partial.to(dev)
        out_parts = car.reduce_residual(pend, r_dev, parts)
        # two-shot (4+ ranks, 256-column chunk groups per owner) or one-shot
        two = world >= 4 and N % (256 * world) == 0
        assert out_parts.shape[0] == (N // 256 if two else N // 1024), (world, N, tuple(out_parts.shape))
        want, want_sq = _rr_reference(all_slabs, all_part, res, S, out_parts.shape[0])
        torch.cuda.synchronize()
        gotr = r_dev.cpu()
        if not torch.equal(gotr, want):
            bad = (gotr != want)
            idx = bad.nonzero()[:4].tolist()
            raise AssertionError((M, N, S, "err", car.error(), "nbad", int(bad.sum()),
                                  [(i, float(gotr[i[0], i[1]]), float(want[i[0], i[1]]), float(res[i[0], i[1]]))
                                   for i in idx]))
        torch.testing.assert_close(out_parts.cpu(), want_sq, rtol=1e-5, atol=1e-3)
        # an all-gather and an all-reduce with other grids in between (epoch consistency)
        lg = torch.full((M, 256), float(rank), dtype=torch.bfloat16, device=dev)
        got = car.all_gather_last(lg)
        torch.cuda.synchronize()
        gv = got.cpu().view(M, world, 256).float()
        assert torch.equal(gv, torch.arange(world, dtype=torch.float32).view(1, world, 1).expand(M, world, 256)), \
            (M, N, S, gv[0, :, 0].tolist(), gv[-1, :, -1].tolist(), car.error())
    # graph replay of the fused collective
    M, N = 8, 4096
    res0 = torch.randn(M, N, generator=g).to(torch.bfloat16)
    part_in = torch.zeros(M, N, dtype=torch.bfloat16, device=dev)
    r_dev = res0.to(dev)
    parts = torch.zeros((N // 256) * M, dtype=torch.float32, device=dev)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        car.reduce_residual(part_in, r_dev, parts)
    torch.cuda.current_stream().wait_stream(s)
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        car.reduce_residual(part_in, r_dev, parts)
    for it in range(3):
        part_in.fill_(float(rank + 1))
        r_dev.copy_(res0.to(dev))
        dist.barrier()
        graph.replay()
        torch.cuda.synchronize()
        inc = torch.tensor(float(sum(r + 1 for r in range(world)))).to(torch.bfloat16).float()
        want = (res0.float() + inc).to(torch.bfloat16)
        assert torch.equal(r_dev.cpu(), want), it
    assert car.error() == 0


def _serving_phase(car, rank, world, dev):
    """parallel/preflight.check_custom_ar_serving on the real kernels: 16 back-to-back fused
    collectives at a decode shape (bf16 partials and fp32 slabs alternating), eager and graph-
    replayed, bit-exact against the locally computed sums; the timed replay reports a per-call time."""
    from polykey_service_amd.parallel import preflight
    car.fused_blocks = 32  # every rank's grid resident at once on the shared GPU
    dist.barrier()
    r = preflight.check_custom_ar_serving(car, rank, world, dev, 64, 4096)
    assert r["checks"] and all(r["checks"].values()), (car.fenced, r)
    assert set(r["checks"]) == {"eager", "graph", "graph_timed"} and r["collective_us"] > 0, r
    # the opt-in forms' preflight checks on the real kernels: column chunks, GEMM push
    dist.barrier()
    c = preflight.check_chunk_form(car, rank, world, dev, 64, 4096, 2)
    assert c == ({"chunks_2": True} if car.chunks_ok(64, 4096, 2) else {}), c
    if not car.fenced:
        dist.barrier()
        p = preflight.check_push_form(car, rank, world, dev, 64, 4096)
        assert p == ({"push": True} if car.push_ok(64, 4096, 64) else {}), p
    assert car.error() == 0


def _carry_phase(car, rank, world, dev):
    """The collective carried by its consumer's launch (kernels/car_gemm.hip):
    residual, norm parts and the consumer's split-K slabs bit-identical to reduce_residual + the
    separate folded-norm projection, across real ranks (small shapes: every rank's grid resident on
    the shared GPU), repeated and graph-replayed (the hand-off counters re-arm themselves)."""
    from polykey_service_amd.ops import gemm
    if not car.carry_ok(8, 256 * world):
        return
    g = torch.Generator().manual_seed(11)
    gr = torch.Generator().manual_seed(200 + rank)
    flow = torch.zeros(gemm.FLOW_WORDS, dtype=torch.int32, device=dev)
    dctx = car.device_ctx()
    for M, N, Nc, S_o, S_c, half in ((8, 256 * world, 512, 2, 4, False), (5, 512 * world, 256, 1, 2, True)):
        K = N
        res0 = (torch.randn(M, N, generator=g) * 2).to(torch.bfloat16).to(dev)
        slabs = torch.randn(S_o * M * N, generator=gr).to(dev)
        w = (torch.randn(Nc, K, generator=g) * 0.05).to(torch.bfloat16).to(dev)
        wp = gemm.pack_weight(w)
        pend = gemm.Partial(slabs, S_o, M, N)
        # reference: the two launches
        r_ref = res0.clone()
        p_ref = torch.zeros((N // 256) * M, dtype=torch.float32, device=dev)
        pv = car.reduce_residual(pend, r_ref, p_ref)
        ws_ref = torch.empty(S_c * M * Nc, dtype=torch.float32, device=dev)
        c_ref = gemm.linear_partial_rowscale(r_ref, w, ws_ref, gemm.RowScale(pv, 1e-5), S=S_c, packed=wp, half=half)
        torch.cuda.synchronize()
        for it in range(3):
            r = res0.clone()
            p = torch.zeros_like(p_ref)
            ws = torch.full((S_c * M * Nc,), float("nan"), device=dev)
            dist.barrier()
            pv2, c = gemm.linear_partial_rowscale_car(dctx, pend, r, p, w, ws, 1e-5, flow, packed=wp, S=S_c, half=half)
            torch.cuda.synchronize()
            assert torch.equal(r, r_ref), ("residual", M, N, it, car.error())
            assert torch.equal(pv2, pv), ("parts", M, N, it)
            assert c.S == c_ref.S and torch.equal(c.view(), c_ref.view()), ("slabs", M, N, it)
            assert int(flow.abs().sum()) == 0, flow.nonzero()[:8].tolist()
    # graph replay of the carried launch
    M, N, Nc = 8, 256 * world, 512
    res0 = torch.randn(M, N, generator=g).to(torch.bfloat16).to(dev)
    r = res0.clone()
    slabs = torch.zeros(2 * M * N, device=dev)
    pend = gemm.Partial(slabs, 2, M, N)
    w = (torch.randn(Nc, N, generator=g) * 0.05).to(torch.bfloat16).to(dev)
    wp = gemm.pack_weight(w)
    p = torch.zeros((N // 256) * M, dtype=torch.float32, device=dev)
    ws = torch.empty(4 * M * Nc, dtype=torch.float32, device=dev)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        gemm.linear_partial_rowscale_car(dctx, pend, r, p, w, ws, 1e-5, flow, packed=wp, S=4)
    torch.cuda.current_stream().wait_stream(s)
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        _, cg = gemm.linear_partial_rowscale_car(dctx, pend, r, p, w, ws, 1e-5, flow, packed=wp, S=4)
    for it in range(3):
        slabs.fill_(float(rank + it))
        r.copy_(res0)
        dist.barrier()
        graph.replay()
        torch.cuda.synchronize()
        inc = torch.tensor(2.0 * sum(r2 + it for r2 in range(world))).to(torch.bfloat16).float()
        assert torch.equal(r, (res0.float() + inc).to(torch.bfloat16)), it
        want = gemm.linear_partial_rowscale(r, w, torch.empty_like(ws), gemm.RowScale(p.view(N // 256, M), 1e-5),
                                            S=4, packed=wp)
        torch.cuda.synchronize()
        assert torch.equal(cg.view(), want.view()), it
    assert car.error() == 0 and int(flow.abs().sum()) == 0


def _overlap_phase(car, rank, world, dev):
    """The fused collective overlapped with its GEMM: the projection as C column-
    chunk GEMMs on the compute stream, each chunk's collective on a side stream behind an event
    after its GEMM (reduce_residual_chunk).  Residual and parts bit-identical to one GEMM + one
    collective, eager and graph-replayed (the side-stream fork / join inside the graph)."""
    from polykey_service_amd.ops import gemm
    car.fused_blocks = 32
    g = torch.Generator().manual_seed(11)
    gr = torch.Generator().manual_seed(2000 + rank)
    M, K, N, C = 64, 1024, 8192, 2
    assert car.chunks_ok(M, N, C)
    res0 = (torch.randn(M, N, generator=g) * 2).to(torch.bfloat16).to(dev)
    x = torch.randn(M, K, generator=gr).to(torch.bfloat16).to(dev)
    w = (torch.randn(N, K, generator=gr) * 0.05).to(torch.bfloat16).to(dev)
    wp = gemm.pack_weight(w)
    ws1 = torch.empty(8 * M * N, dtype=torch.float32, device=dev)
    ws2 = torch.empty_like(ws1)
    np_ = car.nparts(M, N)
    p1 = torch.zeros(np_ * M, dtype=torch.float32, device=dev)
    p2 = torch.zeros_like(p1)
    r1, r2 = res0.clone(), res0.clone()
    cs = torch.cuda.Stream()
    Nc = N // C

    def ref():
        r1.copy_(res0)
        car.reduce_residual(gemm.linear_partial(x, w, ws1, packed=wp, half=True), r1, p1)

    def overlapped():
        r2.copy_(res0)
        main = torch.cuda.current_stream()
        off = 0
        for c in range(C):
            pc = gemm.linear_partial(x, w[c * Nc:(c + 1) * Nc], ws2[off:], packed=wp[c * Nc:(c + 1) * Nc], half=True)
            off += pc.S * M * Nc
            ev = torch.cuda.Event()
            ev.record(main)
            cs.wait_event(ev)
            with torch.cuda.stream(cs):
                car.reduce_residual_chunk(pc, r2, p2, c, C)
        main.wait_stream(cs)

    for it in range(2):
        dist.barrier()
        ref()
        torch.cuda.synchronize()
        dist.barrier()
        overlapped()
        torch.cuda.synchronize()
        assert torch.equal(r1, r2), ("residual", it, car.error())
        assert torch.equal(p1, p2), ("parts", it)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    dist.barrier()
    with torch.cuda.stream(s):
        overlapped()
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    graph = torch.cuda.CUDAGraph()
    dist.barrier()
    with torch.cuda.graph(graph):
        overlapped()
    for it in range(3):
        dist.barrier()
        ref()
        torch.cuda.synchronize()
        dist.barrier()
        graph.replay()
        torch.cuda.synchronize()
        assert torch.equal(r1, r2) and torch.equal(p1, p2), ("graph", it)
    assert car.error() == 0


def _push_phase(car, rank, world, dev):
    """The GEMM epilogue drives the collective (gemm.push_projection): the o / down
    projections' last split of every n-block stores its bf16 tile into the owner rank's slot and
    stamps the owner's push flag; reduce_residual_pushed starts at the reduce-scatter.  Residual and
    parts bit-identical to GEMM + two-shot reduce_residual at the 70B TP=8 per-rank shapes, eager,
    interleaved with other collectives, and graph-replayed."""
    from polykey_service_amd.ops import gemm
    M, N = 64, 8192
    if not car.push_ok(M, N, 64):
        assert world < 4  # the one-shot layout (parts per 1024 columns) stays unpushed
        return
    car.fused_blocks = 32
    tgt = car.push_target()
    assert tgt.rank == rank and tgt.world == world
    g = torch.Generator().manual_seed(13)
    gr = torch.Generator().manual_seed(3000 + rank)
    ctr = torch.zeros(N // 64, dtype=torch.int32, device=dev)
    np_ = car.nparts(M, N)
    assert np_ == N // 256
    for K, down in ((1024, False), (3584, True)):
        res0 = (torch.randn(M, N, generator=g) * 2).to(torch.bfloat16).to(dev)
        x = torch.randn(M, K, generator=gr).to(torch.bfloat16).to(dev)
        w = (torch.randn(N, K, generator=gr) * 0.05).to(torch.bfloat16).to(dev)
        wp = gemm.pack_weight(w)
        ws1 = torch.empty(8 * M * N, dtype=torch.float32, device=dev)
        ws2 = torch.empty_like(ws1)
        p1 = torch.zeros(np_ * M, dtype=torch.float32, device=dev)
        p2 = torch.zeros_like(p1)
        r1, r2 = res0.clone(), res0.clone()

        def ref():
            r1.copy_(res0)
            pend = gemm.linear_down(x, w, ws1, wp) if down else gemm.linear_partial(x, w, ws1, packed=wp, half=True)
            car.reduce_residual(pend, r1, p1)

        def pushed():
            r2.copy_(res0)
            nbc = gemm.push_projection(x, w, ws2, wp, ctr, tgt, down=down)
            car.reduce_residual_pushed(r2, p2, nbc)

        for it in range(2):
            dist.barrier()
            ref()
            torch.cuda.synchronize()
            dist.barrier()
            pushed()
            torch.cuda.synchronize()
            assert car.error() == 0, ("push timeout", K, it)
            assert torch.equal(r1, r2), ("residual", K, it, int((r1 != r2).sum()))
            assert torch.equal(p1, p2), ("parts", K, it)
            assert int(ctr.abs().sum()) == 0, "split-K counters must be left zeroed"
            # another collective in between: the push GEMM reads the shared call epoch
            car.all_reduce(torch.ones(4096, dtype=torch.bfloat16, device=dev))
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        dist.barrier()
        with torch.cuda.stream(s):
            pushed()
        torch.cuda.current_stream().wait_stream(s)
        torch.cuda.synchronize()
        graph = torch.cuda.CUDAGraph()
        dist.barrier()
        with torch.cuda.graph(graph):
            pushed()
        for it in range(3):
            dist.barrier()
            ref()
            torch.cuda.synchronize()
            dist.barrier()
            graph.replay()
            torch.cuda.synchronize()
            assert torch.equal(r1, r2) and torch.equal(p1, p2), ("graph", K, it)
    assert car.error() == 0


@pytest.mark.parametrize("world", [2, 4, 8])
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


def test_loopback_group_runs_every_collective_without_blocking():
    """The one-process stand-in group tools/tp_solo.py --car loopback times the real collective
    kernels with: every form (one-/two-shot all-reduce, all-gather, fused and pushed reduce) runs
    to completion in one process, graph-replayed too, and no wait times out."""
    from polykey_service_amd.ops import gemm
    from polykey_service_amd.parallel.custom_ar import CustomAllReduce
    dev = torch.device("cuda:0")
    car = CustomAllReduce.loopback(0, 8, dev)
    car.set_timeout(2.0)
    try:
        M, N, K = 64, 8192, 1024
        x = torch.randn(M, K, device=dev).to(torch.bfloat16)
        wp = gemm.pack_weight((torch.randn(N, K, device=dev) * 0.05).to(torch.bfloat16))
        ws = torch.empty(8 * M * N, dtype=torch.float32, device=dev)
        res = torch.zeros(M, N, dtype=torch.bfloat16, device=dev)
        parts = torch.zeros((N // 256) * M, dtype=torch.float32, device=dev)
        ctr = torch.zeros(N // 64, dtype=torch.int32, device=dev)

        def chain():
            car.all_reduce(torch.ones(4096, dtype=torch.bfloat16, device=dev), algo=1)
            car.all_reduce(torch.ones(1 << 20, dtype=torch.bfloat16, device=dev), algo=2)
            car.all_gather_last(torch.ones(M, 256, dtype=torch.bfloat16, device=dev))
            car.reduce_residual(gemm.linear_partial(x, wp, ws, packed=wp, half=True), res, parts)
            nbc = gemm.push_projection(x, wp, ws, wp, ctr, car.push_target())
            car.reduce_residual_pushed(res, parts, nbc)

        chain()
        torch.cuda.synchronize()
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            chain()
        torch.cuda.current_stream().wait_stream(s)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            chain()
        for _ in range(3):
            g.replay()
        torch.cuda.synchronize()
        assert car.error() == 0 and int(ctr.abs().sum()) == 0
    finally:
        car.close()


@pytest.mark.parametrize("consumer", ["gate_up", "qkv"])
def test_carried_collective_at_70b_tp8_shapes_on_loopback(consumer):
    """The carried launch at the 70B TP=8 rank's real shapes (64 rows, hidden 8192; gate_up 7168 x
    8192 split 4 after o, QKV 1280 x 8192 half-split after down) on the one-process loopback group:
    every workgroup of the real grid runs (256 collective items + 224 / 160 consumer tiles), the
    results equal the two launches bit for bit, the hand-off counters re-arm."""
    from polykey_service_amd.ops import gemm
    from polykey_service_amd.parallel.custom_ar import CustomAllReduce
    dev = torch.device("cuda:0")
    car = CustomAllReduce.loopback(0, 8, dev)
    car.set_timeout(5.0)
    try:
        M, N = 64, 8192
        Nc, S_c, half = (7168, 4, False) if consumer == "gate_up" else (1280, None, True)
        g = torch.Generator(device=dev).manual_seed(3)
        res0 = (torch.randn(M, N, device=dev, generator=g) * 2).to(torch.bfloat16)
        slabs = torch.randn(2 * M * N, device=dev, generator=g)
        pend = gemm.Partial(slabs, 2, M, N)
        w = (torch.randn(Nc, N, device=dev, generator=g) * 0.02).to(torch.bfloat16)
        wp = gemm.pack_weight(w)
        S_real, _ = gemm._rowscale_tiling(Nc, N, M, wp, half, S_c)
        assert car.carry_ok(M, N)
        r_ref = res0.clone()
        p_ref = torch.zeros((N // 256) * M, dtype=torch.float32, device=dev)
        pv = car.reduce_residual(pend, r_ref, p_ref)
        c_ref = gemm.linear_partial_rowscale(r_ref, w, torch.empty(S_real * M * Nc, device=dev), gemm.RowScale(pv, 1e-5),
                                             S=S_c, packed=wp, half=half)
        flow = torch.zeros(gemm.FLOW_WORDS, dtype=torch.int32, device=dev)
        dctx = car.device_ctx()
        for _ in range(3):
            r = res0.clone()
            p = torch.zeros_like(p_ref)
            pv2, c = gemm.linear_partial_rowscale_car(dctx, pend, r, p, w, torch.empty(S_real * M * Nc, device=dev),
                                                      1e-5, flow, packed=wp, S=S_c, half=half)
            torch.cuda.synchronize()
            assert torch.equal(r, r_ref) and torch.equal(pv2, pv)
            assert torch.equal(c.view(), c_ref.view())
        assert car.error() == 0 and int(flow.abs().sum()) == 0
    finally:
        car.close()
