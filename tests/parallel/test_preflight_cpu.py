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
        self.forms = set()

    def supports_gather(self, x):
        return True

    def all_gather_last(self, x):
        parts = [torch.empty_like(x) for _ in range(self.world)]
        dist.all_gather(parts, x.contiguous(), group=self.g)
        return torch.cat(parts, -1)

    def supports_reduce_residual(self, M, N):
        return N % 1024 == 0

    def nparts(self, M, N):
        # csrc/comm/custom_allreduce.hip pk_car_reduce_residual_nparts: two-shot (parts per 256
        # columns) from 4 ranks when 256-column chunk groups tile N, else one-shot (per 1024)
        return N // 256 if self.world >= 4 and N % (256 * self.world) == 0 else N // 1024

    def reduce_residual(self, pending, residual, parts):
        s = pending.float().clone()
        dist.all_reduce(s, group=self.g)
        residual.copy_((residual.float() + s).to(residual.dtype))
        M, N = residual.shape
        n = self.nparts(M, N)
        assert parts.numel() >= n * M  # the real reduce_residual's check
        pv = parts.view(-1)[: n * M].view(n, M)
        pv.copy_(residual.float().view(M, n, N // n).pow(2).sum(-1).t())
        self.forms.add("2shot" if N // n == 256 else "1shot")
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
                "car_closed": car.closed, "forms": sorted(car.forms)}, f"{out}.{rank}")
    st.rccl_tp = st.custom_ar = None
    destroy_parallel()


class SlowComm(GlooComm):
    """A collective whose peer arrives late (a hung RCCL call until the watchdog aborts it)."""

    aborted = False

    def all_reduce(self, x, op="sum", out=None):
        import time
        time.sleep(4.0)
        return super().all_reduce(x, op, out)

    def abort(self):
        SlowComm.aborted = True


def _hang_worker(rank, world, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank), POLYKEY_PREFLIGHT="0")
    from polykey_service_amd.parallel import preflight
    from polykey_service_amd.parallel.state import destroy_parallel, init_parallel
    preflight.HANG_S = 1.0
    st = init_parallel(tp=world, device="cpu", backend="gloo")
    st.rccl_tp = (SlowComm if rank == 1 else GlooComm)(st.tp_cpu_group, world)
    st.custom_ar = FakeCar(st.tp_cpu_group, world)
    lines = []
    rep = preflight.run(st, emit=lines.append)
    torch.save({"report": rep, "lines": lines, "rccl": st.rccl_tp is not None, "car": st.custom_ar is not None,
                "aborted": SlowComm.aborted}, f"{out}.{rank}")
    st.rccl_tp = st.custom_ar = None
    destroy_parallel()


def test_preflight_watchdog_aborts_a_hung_check_and_disables_it(tmp_path):
    """a direct-RCCL check that does not return within HANG_S (rank 1's
    all-reduce stalls; rank 0 waits in it) is reported as hung in a line emitted at once, aborted
    (ncclCommAbort's stand-in), failed, and disabled on BOTH ranks; the healthy path stays."""
    out = str(tmp_path / "pf")
    mp.start_processes(_hang_worker, args=(2, _port(), out), nprocs=2, join=True, start_method="spawn")
    for r in range(2):
        d = torch.load(f"{out}.{r}", weights_only=True)
        rep = d["report"]
        assert rep["hung"] == ["rccl_tp"] and "hung" in rep["checks"]["rccl_tp"]["error"], rep
        assert rep["disabled"] == ["rccl_tp"] and not d["rccl"] and d["car"], rep
        assert d["aborted"] == (r == 1)
        # the first line is the watchdog's (emitted while the check was still stuck)
        assert json.loads(d["lines"][0])["hung"] == ["rccl_tp"]


def test_preflight_watchdog_exits_when_the_abort_does_not_unblock(tmp_path):
    """A check that stays stuck after its abort: the process prints the report line with "exit"
    and leaves with HANG_EXIT instead of hanging the job."""
    import subprocess
    import sys
    code = ("import threading, json\n"
            "from polykey_service_amd.parallel import preflight as p\n"
            "rep = {'event': 'multi_gpu_preflight'}\n"
            "p._guarded('rccl_tp', lambda: threading.Event().wait(), lambda: None, rep,\n"
            "           lambda s: print(s, flush=True), hang_s=0.5, grace_s=0.5)\n"
            "print('unreachable')\n")
    root = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    r = subprocess.run([sys.executable, "-c", code], cwd=root, capture_output=True, text=True, timeout=60)
    from polykey_service_amd.parallel.preflight import HANG_EXIT
    assert r.returncode == HANG_EXIT, (r.returncode, r.stdout, r.stderr)
    lines = [json.loads(l) for l in r.stdout.splitlines() if l.startswith("{")]
    assert lines[0]["hung"] == ["rccl_tp"] and "still hung" in lines[-1]["exit"]
    assert "unreachable" not in r.stdout


def _car_worker(rank, world, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank), POLYKEY_PREFLIGHT="0")
    from polykey_service_amd.parallel import preflight
    from polykey_service_amd.parallel.state import destroy_parallel, init_parallel
    st = init_parallel(tp=world, device="cpu", backend="gloo")
    car = st.custom_ar = FakeCar(st.tp_cpu_group, world)
    rep = preflight.run(st, paths=("custom_ar",), emit=lambda s: None)
    torch.save({"report": rep, "car": st.custom_ar is not None, "forms": sorted(car.forms)}, f"{out}.{rank}")
    st.custom_ar = None
    destroy_parallel()


@pytest.mark.parametrize("world", [4, 8])
def test_preflight_checks_both_forms_of_the_fused_collective(tmp_path, world):
    """at TP=4 the 1024-column check took the two-shot form with parts sized for the
    one-shot one, failed its own assert and disabled the custom all-reduce on every rank; at TP=8
    the two-shot form a 70B decode step uses was never checked.  Both forms now run, each with
    parts sized by car.nparts, and the path stays enabled."""
    out = str(tmp_path / "pf")
    mp.start_processes(_car_worker, args=(world, _port(), out), nprocs=world, join=True, start_method="spawn")
    for r in range(world):
        d = torch.load(f"{out}.{r}", weights_only=True)
        chk = d["report"]["checks"]["custom_ar"]
        assert chk["ok"] and chk["group_ok"] and d["car"], chk
        assert d["forms"] == ["1shot", "2shot"] if world == 8 else d["forms"] == ["2shot"], d["forms"]
        names = {k for k in chk if k.startswith("reduce_residual")}
        assert names == ({"reduce_residual_1shot_1024", "reduce_residual_2shot_2048"} if world == 8
                         else {"reduce_residual_2shot_1024"}), names


@pytest.mark.parametrize("faulty_rank", [-1, 1])
def test_preflight_disables_a_faulty_collective_on_every_rank(tmp_path, faulty_rank):
    out = str(tmp_path / "pf")
    mp.start_processes(_worker, args=(2, _port(), out, faulty_rank), nprocs=2, join=True, start_method="spawn")
    res = [torch.load(f"{out}.{r}", weights_only=True) for r in range(2)]
    for r, d in enumerate(res):
        rep = d["report"]
        assert rep["checks"]["custom_ar"]["ok"] and d["car"] and not d["car_closed"], rep
        assert set(rep["checks"]["custom_ar"]) >= {"all_gather_1shot", "reduce_residual_1shot_1024"}
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


class StaleCar(FakeCar):
    """The fused collective of FakeCar with the protocol switch of custom_ar.CustomAllReduce; on
    ``stale_rank`` the 11th call of 16 (in the protocols listed in ``stale_in``) reads the peer
    sum of the PREVIOUS call -- a slot served stale, the failure a fence-free protocol could
    show on real xGMI."""

    def __init__(self, group, world, stale_rank, stale_in):
        super().__init__(group, world)
        self.stale_rank, self.stale_in = stale_rank, stale_in
        self.fenced, self.calls, self.prev, self.failed, self.switched = False, 0, None, False, []

    def set_fenced(self, on):
        self.fenced = bool(on)
        self.calls = 0
        self.switched.append(bool(on))

    def error(self):
        return 0

    def fail(self):
        self.failed = True

    def reduce_residual(self, pending, residual, parts):
        src = pending.view().sum(0) if hasattr(pending, "view") and not isinstance(pending, torch.Tensor) \
            else pending.float()
        s = src.float().clone()
        dist.all_reduce(s, group=self.g)
        self.calls += 1
        proto = "fenced" if self.fenced else "fence-free"
        if (dist.get_rank(self.g) == self.stale_rank and self.calls == 11 and proto in self.stale_in
                and self.prev is not None):
            s = self.prev  # the previous call's slot contents
        self.prev = s
        residual.copy_((residual.float() + s.to(torch.bfloat16).float()).to(residual.dtype))
        M, N = residual.shape
        n = self.nparts(M, N)
        pv = parts.view(-1)[: n * M].view(n, M)
        pv.copy_(residual.float().view(M, n, N // n).pow(2).sum(-1).t())
        return pv


def _serving_worker(rank, world, port, out, stale_in):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank), POLYKEY_PREFLIGHT="0")
    from polykey_service_amd.parallel import preflight
    from polykey_service_amd.parallel.state import destroy_parallel, init_parallel
    st = init_parallel(tp=world, device="cpu", backend="gloo")
    car = st.custom_ar = StaleCar(st.tp_cpu_group, world, stale_rank=1, stale_in=stale_in)
    lines = []
    rep = preflight.run(st, paths=("custom_ar_serving",), emit=lines.append, serving=(8, 2048))
    torch.save({"report": rep, "lines": lines, "car": st.custom_ar is not None, "closed": car.closed,
                "switched": car.switched, "fenced": car.fenced}, f"{out}.{rank}")
    st.custom_ar = None
    destroy_parallel()


@pytest.mark.parametrize("stale_in", [(), ("fence-free",), ("fence-free", "fenced")])
def test_serving_preflight_catches_a_stale_slot_and_falls_back(tmp_path, stale_in):
    """VERDICT r5 item 2 / ADVICE r5: the fused collective at serving shape, 16 back-to-back calls.
    A stale slot read on call 11 of 16 on ONE rank fails the fence-free check on that rank; the
    group agrees, switches to the fenced protocol on BOTH ranks and checks again.  If the fenced
    protocol reads stale too, the custom collectives are disabled on both ranks (RCCL takes over);
    a clean group keeps the fence-free protocol.  The report line carries the per-call time."""
    out = str(tmp_path / "pf")
    mp.start_processes(_serving_worker, args=(2, _port(), out, stale_in), nprocs=2, join=True, start_method="spawn")
    for r in range(2):
        d = torch.load(f"{out}.{r}", weights_only=True)
        rep = d["report"]
        assert rep["serving_shape"] == [8, 2048]
        if not stale_in:
            assert rep["checks"]["custom_ar_serving"]["ok"] and rep["car_protocol"] == "fence-free", rep
            assert d["car"] and d["switched"] == [] and rep["disabled"] == []
            assert rep["collective_us"]["custom_ar_serving"] > 0
            continue
        first = rep["checks"]["custom_ar_serving"]
        assert first["ok"] == (r != 1) and not first["group_ok"], rep  # only rank 1 saw the stale read
        assert d["switched"] == [True] and rep["car_protocol"] == "fenced"  # both ranks switched
        fenced = rep["checks"]["custom_ar_serving_fenced"]
        if stale_in == ("fence-free",):
            assert fenced["ok"] and fenced["group_ok"] and d["car"] and not d["closed"] and rep["disabled"] == []
        else:
            assert not fenced["group_ok"] and not d["car"] and d["closed"], rep
            assert rep["disabled"] == ["custom_ar_serving_fenced"]
    line = json.loads(torch.load(f"{out}.0", weights_only=True)["lines"][-1])
    assert line["event"] == "multi_gpu_preflight" and "collective_us" in line


class ChunkCar(StaleCar):
    """StaleCar plus the column-chunk form; ``bad_chunk`` >= 0 drops that chunk's peer sum on rank 1."""

    def __init__(self, group, world, bad_chunk):
        super().__init__(group, world, stale_rank=-1, stale_in=())
        self.bad_chunk = bad_chunk

    def chunks_ok(self, M, N, chunks):
        return N % (1024 * chunks) == 0

    def reduce_residual_chunk(self, pending, residual, parts, chunk, chunks):
        M, N = residual.shape
        Nc = N // chunks
        s = pending.view().sum(0).float().clone()
        dist.all_reduce(s, group=self.g)
        if chunk == self.bad_chunk and dist.get_rank(self.g) == 1:
            s.zero_()
        cols = slice(chunk * Nc, (chunk + 1) * Nc)
        residual[:, cols] = (residual[:, cols].float() + s.to(torch.bfloat16).float()).to(residual.dtype)
        n = self.nparts(M, N)
        w = N // n
        pv = parts.view(-1)[: n * M].view(n, M)
        pv[chunk * (Nc // w):(chunk + 1) * (Nc // w)] = residual[:, cols].float().view(M, Nc // w, w).pow(2).sum(-1).t()


def _chunk_worker(rank, world, port, out, bad_chunk):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank), POLYKEY_PREFLIGHT="0")
    from polykey_service_amd.ops import gemm
    from polykey_service_amd.parallel import preflight
    from polykey_service_amd.parallel.state import destroy_parallel, init_parallel
    gemm.TP_DECODE_CHUNKS = 2
    st = init_parallel(tp=world, device="cpu", backend="gloo")
    st.custom_ar = ChunkCar(st.tp_cpu_group, world, bad_chunk)
    rep = preflight.run(st, paths=("custom_ar_serving",), emit=lambda s: None, serving=(8, 2048))
    torch.save({"report": rep, "chunks": gemm.TP_DECODE_CHUNKS, "car": st.custom_ar is not None}, f"{out}.{rank}")
    st.custom_ar = None
    destroy_parallel()


@pytest.mark.parametrize("bad_chunk", [-1, 1])
def test_serving_preflight_checks_the_chunk_form(tmp_path, bad_chunk):
    """with POLYKEY_TP_DECODE_CHUNKS > 1 the column-chunk collective is checked at serving
    shape too; a wrong chunk on one rank turns the chunked chain off on both ranks and keeps the
    plain fused collective."""
    out = str(tmp_path / "pf")
    mp.start_processes(_chunk_worker, args=(2, _port(), out, bad_chunk), nprocs=2, join=True, start_method="spawn")
    for r in range(2):
        d = torch.load(f"{out}.{r}", weights_only=True)
        chk = d["report"]["checks"]["tp_decode_chunks"]
        assert d["car"] and d["report"]["checks"]["custom_ar_serving"]["group_ok"]
        if bad_chunk < 0:
            assert chk["ok"] and chk["group_ok"] and d["chunks"] == 2, chk
        else:
            assert chk["ok"] == (r != 1) and not chk["group_ok"] and d["chunks"] == 1, chk
            assert d["report"]["disabled"] == ["tp_decode_chunks"]
