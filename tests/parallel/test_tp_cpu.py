"""Tensor / expert / sequence parallel correctness on CPU with gloo at 2, 4 and 8 ranks: the
sharded model must reproduce the single-rank model (same random-init weights, shards sliced from
the full tensors).  ``tiny-llama-g8`` has the per-rank shape of Llama-3-70B at TP=8 (one KV head
per rank, GQA group 8, padded vocab shards) and ``tiny-mixtral-e8`` Mixtral's 8 experts (one per
rank at EP=8), so the north-star configs' rank counts run here (BASELINE.json:10-11)."""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

PROMPTS = [[1, 5, 6, 7, 8, 9], [1] + list(range(20, 60)), [1, 2]]


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _engine(model, st, **kw):
    from polykey_service_amd.engine import EngineConfig, LLMEngine
    return LLMEngine(EngineConfig(model=model, max_num_seqs=8, max_num_batched_tokens=128, max_model_len=256,
                                  hip_graphs=False, device="cpu", **kw), st)


def _first_step_logits_and_tokens(eng):
    from polykey_service_amd.engine import SamplingParams
    eng.runner.keep_logits = True
    seqs = [eng.add_request(p, SamplingParams(max_tokens=4)) for p in PROMPTS]
    eng.step()
    logits = eng.runner.last_logits.float().clone()
    while eng.has_unfinished():
        eng.step()
    return logits, [s.output_ids for s in seqs]


def _worker(rank, world, port, model, ep, out_path, sp=False):  # noqa: PLR0913
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    torch.set_num_threads(max(1, 8 // world))
    from polykey_service_amd.models import llama
    llama.SP_MIN_TOKENS = 1 if sp else 1 << 30  # sp: every step (49-token prefill: padded rows) runs SP
    from polykey_service_amd.parallel.state import destroy_parallel, init_parallel
    st = init_parallel(tp=world, ep=ep, device="cpu", backend="gloo")
    eng = _engine(model, st)
    if st.tp_rank == 0:
        logits, toks = _first_step_logits_and_tokens(eng)
        eng.runner.stop_workers()
        torch.save({"logits": logits, "tokens": toks}, out_path)
    else:
        eng.runner.worker_loop()
    destroy_parallel()


@pytest.mark.parametrize("model,world,ep,sp", [
    ("tiny-llama-gqa4", 2, 1, False), ("tiny-mixtral", 2, 1, False), ("tiny-mixtral", 2, 2, False),
    ("tiny-llama-gqa4", 2, 1, True), ("tiny-mixtral", 2, 2, True),
    # 70B TP=8 shape: 8-way all-reduces, one KV head per rank, 126-row vocab shards
    ("tiny-llama-g8", 4, 1, False), ("tiny-llama-g8", 8, 1, False), ("tiny-llama-g8", 8, 1, True),
    # Mixtral at 8 ranks: tensor-parallel experts (EP=1) and one expert per rank (EP=8)
    ("tiny-mixtral-e8", 8, 1, False), ("tiny-mixtral-e8", 8, 8, False), ("tiny-mixtral-e8", 8, 8, True)])
def test_tp_matches_tp1(tmp_path, model, world, ep, sp):
    """``sp``: sequence-parallel steps (token-sharded residual, reduce-scatter / all-gather)."""
    from polykey_service_amd.parallel.state import ParallelState
    ref_logits, ref_toks = _first_step_logits_and_tokens(_engine(model, ParallelState()))
    out = str(tmp_path / "tp.pt")
    mp.start_processes(_worker, args=(world, _free_port(), model, ep, out, sp), nprocs=world, join=True,
                       start_method="spawn")
    got = torch.load(out, weights_only=True)
    # bf16 row-parallel partials are rounded per rank before the all-reduce: ~1 bf16 ulp noise
    torch.testing.assert_close(got["logits"], ref_logits, atol=1e-1, rtol=5e-2)
    _same_first_tokens(got["tokens"], ref_toks, ref_logits)


def _same_first_tokens(got_toks, ref_toks, ref_logits, tie=0.1):
    """First (prefill) tokens equal, except where the reference itself has a near-tie (random
    weights: two logits within bf16 noise of each other may flip under a different reduction)."""
    for row, (g, r) in enumerate(zip(got_toks, ref_toks)):
        if g[0] != r[0]:
            lg = ref_logits[row].float()
            assert lg[g[0]] >= lg.max() - tie, (row, g[0], r[0], float(lg[g[0]]), float(lg.max()))


def _comm_worker(rank, world, port, out_path):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    from polykey_service_amd.parallel import comm
    from polykey_service_amd.parallel.state import destroy_parallel, init_parallel
    init_parallel(tp=world, device="cpu", backend="gloo")
    x = torch.full((2, 3), float(rank + 1))
    ar = comm.tp_all_reduce(x.clone())
    ag = comm.tp_all_gather_last(torch.arange(3, dtype=torch.float32).view(1, 3) + 10 * rank)
    # all-to-all: rank r sends (r+1) rows to every peer
    send = torch.full((world * (rank + 1), 2), float(rank))
    cnt = comm.tp_all_to_all_counts(torch.full((world,), rank + 1, dtype=torch.int64))
    recv = comm.tp_all_to_all(send, cnt.tolist(), [rank + 1] * world)
    obj = comm.tp_broadcast_object({"step": 7} if rank == 0 else None)
    # sequence-parallel layout: 7 rows padded to 8 (2 chunks x 2 ranks x 2 rows)
    lay = comm.SPLayout(7, chunks=2)
    full = torch.arange(7 * 2, dtype=torch.float32).view(7, 2) * (rank + 1)
    shard = comm.sp_reduce_scatter(full, lay)
    back = comm.sp_all_gather(shard, lay)
    twice = comm.sp_all_gather(shard, lay, comm.RowsFn(lambda r, o: torch.mul(r, 2, out=o), 2))
    torch.save({"ar": ar, "ag": ag, "recv": recv, "obj": obj, "shard": shard, "back": back, "twice": twice},
               f"{out_path}.{rank}")
    destroy_parallel()


@pytest.mark.parametrize("world", [2, 4, 8])
def test_collectives_gloo(tmp_path, world):
    out = str(tmp_path / "c")
    mp.start_processes(_comm_worker, args=(world, _free_port(), out), nprocs=world, join=True, start_method="spawn")
    summed = torch.arange(14, dtype=torch.float32).view(7, 2) * (world * (world + 1) // 2)
    Tp = (7 + 2 * world - 1) // (2 * world) * (2 * world)
    padded = torch.cat([summed, torch.zeros(Tp - 7, 2)])
    Tc = Tp // 2
    for r in range(world):
        d = torch.load(f"{out}.{r}", weights_only=True)
        assert torch.equal(d["ar"], torch.full((2, 3), float(world * (world + 1) // 2)))
        assert d["ag"].tolist() == [[float(10 * q + j) for q in range(world) for j in range(3)]]
        assert d["recv"][:, 0].tolist() == [float(q) for q in range(world) for _ in range(q + 1)]
        assert d["obj"] == {"step": 7}
        # rank r holds rows [c*Tc + r*Tc/world, +Tc/world) of chunk c
        per = Tc // world
        want = torch.cat([padded[c * Tc + r * per:c * Tc + (r + 1) * per] for c in range(2)])
        assert torch.equal(d["shard"], want)
        assert torch.equal(d["back"], summed) and torch.equal(d["twice"], 2 * summed)


def _a2a_worker(rank, world, port, out_path):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    from polykey_service_amd.ops import gemm
    from polykey_service_amd.parallel.ep import moe_all_to_all
    from polykey_service_amd.parallel.state import destroy_parallel, init_parallel
    init_parallel(tp=1, ep=world, device="cpu", backend="gloo")
    g = torch.Generator().manual_seed(1)
    E, H, I, k = 4, 256, 256, 2
    router = (torch.randn(E, H, generator=g) * 0.2).to(torch.bfloat16)
    w13 = torch.stack([gemm.interleave_gate_up((torch.randn(I, H, generator=g) * 0.05).to(torch.bfloat16),
                                               (torch.randn(I, H, generator=g) * 0.05).to(torch.bfloat16))
                       for _ in range(E)])
    w2 = (torch.randn(E, H, I, generator=g) * 0.05).to(torch.bfloat16)
    x = torch.randn(12, H, generator=g).to(torch.bfloat16)
    per = E // world
    mine = x[rank * 6:(rank + 1) * 6]
    y = moe_all_to_all(mine, router, w13[rank * per:(rank + 1) * per], w2[rank * per:(rank + 1) * per], k)
    torch.save({"y": y, "x": x, "router": router, "w13": w13, "w2": w2}, f"{out_path}.{rank}")
    destroy_parallel()


def test_moe_all_to_all_matches_dense(tmp_path):
    from polykey_service_amd.ops.moe import fused_moe_reference
    out = str(tmp_path / "a2a")
    mp.start_processes(_a2a_worker, args=(2, _free_port(), out), nprocs=2, join=True, start_method="spawn")
    d0, d1 = torch.load(f"{out}.0", weights_only=True), torch.load(f"{out}.1", weights_only=True)
    y = torch.cat([d0["y"], d1["y"]]).float()
    ref = fused_moe_reference(d0["x"], d0["router"], d0["w13"], d0["w2"], 2)
    torch.testing.assert_close(y, ref, atol=3e-2, rtol=3e-2)


# DP attention + EP: each rank serves its own prompts; ranks 2.. of the 8-rank case get none
# (they only serve the others' expert rows), and rank 0 generates longer, so every other rank
# keeps joining its MoE all-to-alls after finishing its own requests.
DPEP_PROMPTS = {0: [[1, 5, 6, 7, 8, 9], [1, 2]], 1: [[1] + list(range(20, 60))], 3: [[1, 3, 3, 7]]}


def _dpep_max_tokens(rank):
    return 6 if rank == 0 else 3


def _dpep_worker(rank, world, port, model, out_path):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    torch.set_num_threads(max(1, 8 // world))
    from polykey_service_amd.engine import SamplingParams
    from polykey_service_amd.parallel.state import destroy_parallel, init_parallel
    st = init_parallel(tp=1, ep=world, device="cpu", backend="gloo")
    assert st.dp_attention and st.ep_rank == rank
    eng = _engine(model, st)
    eng.runner.keep_logits = True
    prompts = DPEP_PROMPTS.get(rank, [])
    seqs = [eng.add_request(p, SamplingParams(max_tokens=_dpep_max_tokens(rank))) for p in prompts]
    eng.step()
    logits = eng.runner.last_logits.float().clone() if prompts else None
    while eng.any_unfinished():
        eng.step()
    torch.save({"logits": logits, "tokens": [s.output_ids for s in seqs],
                "idle": eng.runner.stats.get("idle_steps", 0)}, f"{out_path}.{rank}")
    destroy_parallel()


@pytest.mark.parametrize("model,world", [("tiny-mixtral", 2), ("tiny-mixtral-e8", 8)])
def test_dp_attention_expert_all_to_all_matches_tp1(tmp_path, model, world):
    """Mixtral with DP attention + EP (one expert per rank at 8): every rank's first-step logits
    and first tokens equal a single-rank engine's on the same prompts."""
    from polykey_service_amd.engine import SamplingParams
    from polykey_service_amd.parallel.state import ParallelState
    out = str(tmp_path / "dpep")
    mp.start_processes(_dpep_worker, args=(world, _free_port(), model, out), nprocs=world, join=True,
                       start_method="spawn")
    ref_eng = _engine(model, ParallelState())
    for r in range(world):
        d = torch.load(f"{out}.{r}", weights_only=True)
        prompts = DPEP_PROMPTS.get(r, [])
        if not prompts:
            assert d["tokens"] == [] and d["idle"] > 0  # served the other ranks' rows only
            continue
        ref_eng.runner.keep_logits = True
        seqs = [ref_eng.add_request(p, SamplingParams(max_tokens=_dpep_max_tokens(r))) for p in prompts]
        ref_eng.step()
        ref_logits = ref_eng.runner.last_logits.float().clone()
        while ref_eng.has_unfinished():
            ref_eng.step()
        torch.testing.assert_close(d["logits"], ref_logits, atol=1e-1, rtol=5e-2)
        assert [t[0] for t in d["tokens"]] == [s.output_ids[0] for s in seqs]
        assert [len(t) for t in d["tokens"]] == [_dpep_max_tokens(r)] * len(prompts)
