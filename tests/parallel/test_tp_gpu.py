"""Tensor parallelism on the GPU code path with 2 ranks sharing one MI355X (gloo carries the
collectives that RCCL would across GPUs; the one-shot IPC all-reduce kernel carries the TP
all-reduces; prefill row-parallel projections take the chunked comm-stream overlap path):
TP=2 must reproduce TP=1 (same random-init weights)."""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

PROMPTS = [[1, 5, 6, 7, 8, 9], [1] + list(range(20, 60)), [1, 2]]


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _engine(model, st):
    from polykey_service_amd.engine import EngineConfig, LLMEngine
    return LLMEngine(EngineConfig(model=model, max_num_seqs=8, max_num_batched_tokens=128, max_model_len=256,
                                  hip_graphs=False, device="cuda:0"), st)


def _run(eng):
    from polykey_service_amd.engine import SamplingParams
    eng.runner.keep_logits = True
    seqs = [eng.add_request(p, SamplingParams(max_tokens=4)) for p in PROMPTS]
    eng.step()
    prefill = eng.runner.last_logits.float().cpu().clone()
    eng.step()  # first decode step (skinny GEMMs + fused TP collective)
    logits = eng.runner.last_logits.float().cpu().clone()
    while eng.has_unfinished():
        eng.step()
    return (prefill, logits), [s.output_ids for s in seqs]


def _compare(got_logits, got_toks, ref_logits, ref_toks):
    """Prefill logits close; first tokens equal unless the reference has a near-tie (random
    weights); first-decode-step logits close on every row that decoded the same token."""
    (gp, gd), (rp, rd) = got_logits, ref_logits
    torch.testing.assert_close(gp, rp, atol=1e-1, rtol=5e-2)
    same = []
    for row, (g, r) in enumerate(zip(got_toks, ref_toks)):
        if g[0] == r[0]:
            same.append(row)
        else:
            assert float(rp[row, g[0]]) >= float(rp[row].max()) - 0.1, (row, g[0], r[0])
    assert same, "no row decoded the reference's first token"
    torch.testing.assert_close(gd[same], rd[same], atol=1e-1, rtol=5e-2)


def _worker(rank, port, model, out_path, sp=False):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE="2",
                      LOCAL_RANK="0", POLYKEY_CUSTOM_AR="force",
                      # sp: the 49-token prefill runs sequence-parallel with 2 comm-stream chunks
                      POLYKEY_SP_MIN_TOKENS="16" if sp else "100000")
    from polykey_service_amd.parallel import comm
    from polykey_service_amd.parallel.state import destroy_parallel, init_parallel
    comm.OVERLAP_MIN_ROWS = 8  # the short prefills take the chunk-overlapped row-parallel path
    st = init_parallel(tp=2, device="cuda", backend="gloo")
    assert st.custom_ar is not None, "custom all-reduce did not come up"
    eng = _engine(model, st)
    if st.tp_rank == 0:
        logits, toks = _run(eng)
        eng.runner.stop_workers()
        torch.save({"logits": logits, "tokens": toks, "car_err": st.custom_ar.error()}, out_path)
    else:
        eng.runner.worker_loop()
    destroy_parallel()


@pytest.mark.parametrize("model,sp", [("tiny-llama-gqa4", False), ("tiny-mixtral", False),
                                      ("tiny-llama-gqa4", True), ("tiny-mixtral", True)])
def test_tp2_on_gpu_matches_tp1(tmp_path, model, sp, monkeypatch):
    from polykey_service_amd.parallel.state import ParallelState
    # like for like: TP = 1 and TP = 2 both fold the RMSNorm weights into their decode
    # projections (TP = 2 ends each row-parallel projection in the fused IPC collective)
    ref_logits, ref_toks = _run(_engine(model, ParallelState(device=torch.device("cuda:0"))))
    out = str(tmp_path / "tp.pt")
    mp.start_processes(_worker, args=(_port(), model, out, sp), nprocs=2, join=True, start_method="spawn")
    got = torch.load(out, weights_only=True)
    assert got["car_err"] == 0
    # logits agree to bf16 noise (row-parallel partials are rounded per rank)
    _compare(got["logits"], got["tokens"], ref_logits, ref_toks)


def _engine2(model, st, graphs):
    from polykey_service_amd.engine import EngineConfig, LLMEngine
    return LLMEngine(EngineConfig(model=model, max_num_seqs=8, max_num_batched_tokens=128, max_model_len=256,
                                  hip_graphs=graphs, device="cuda:0", overlap=graphs), st)


def _run_greedy(eng, max_tokens=8):
    from polykey_service_amd.engine import SamplingParams
    seqs = [eng.add_request(p, SamplingParams(max_tokens=max_tokens, ignore_eos=True)) for p in PROMPTS]
    while eng.has_unfinished():
        eng.step()
    return [s.output_ids for s in seqs], dict(eng.runner.stats), eng.continuation_steps


def _graph_worker(rank, port, model, out_path):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE="2",
                      LOCAL_RANK="0", POLYKEY_CUSTOM_AR="force")
    from polykey_service_amd.parallel.state import destroy_parallel, init_parallel
    st = init_parallel(tp=2, device="cuda", backend="gloo")
    assert st.custom_ar is not None, "custom all-reduce did not come up"
    eager = _engine2(model, st, graphs=False)   # same TP group, same weights, no graphs
    graphed = _engine2(model, st, graphs=True)  # decode graphs + pipelined continuations
    assert graphed.runner.graphs, "no decode graphs captured"
    if st.tp_rank == 0:
        want, _, _ = _run_greedy(eager)
        eager.runner.stop_workers()
        toks, stats, cont = _run_greedy(graphed)
        graphed.runner.stop_workers()
        torch.save({"tokens": toks, "eager": want, "graph_steps": stats["graph_steps"], "cont": cont,
                    "car_err": st.custom_ar.error()}, out_path)
    else:
        eager.runner.worker_loop()
        graphed.runner.worker_loop()
        torch.save({"worker_steps": graphed.runner.stats["steps"]}, out_path + ".w")
    destroy_parallel()


@pytest.mark.parametrize("model", ["tiny-llama-gqa4", "tiny-mixtral"])
def test_tp2_hip_graphs_with_continuations(tmp_path, model):
    """TP decode inside HIP graphs: every collective of the captured step is an IPC kernel (one-shot
    all-reduce, LM-head all-gather), the worker takes steps from the shared-memory ring without a
    GPU sync, and pipelined decode continuations run on both ranks.  The graphed, pipelined TP=2
    engine must generate exactly the tokens of the eager TP=2 engine (same kernels, same sums);
    the prefill token must also match TP=1."""
    from polykey_service_amd.parallel.state import ParallelState
    ref, _, _ = _run_greedy(_engine2(model, ParallelState(device=torch.device("cuda:0")), graphs=False))
    out = str(tmp_path / "tpg.pt")
    mp.start_processes(_graph_worker, args=(_port(), model, out), nprocs=2, join=True, start_method="spawn")
    got = torch.load(out, weights_only=True)
    wk = torch.load(out + ".w", weights_only=True)
    assert got["car_err"] == 0
    assert got["graph_steps"] > 0 and got["cont"] > 0, got
    assert wk["worker_steps"] >= got["graph_steps"]
    assert got["tokens"] == got["eager"]
    assert [t[0] for t in got["tokens"]] == [t[0] for t in ref]


DPEP_PROMPTS = {0: [[1, 5, 6, 7, 8, 9], [1, 2]], 1: [[1] + list(range(20, 60))]}


def _dpep_worker(rank, port, model, out_path):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE="2",
                      LOCAL_RANK="0")
    from polykey_service_amd.engine import SamplingParams
    from polykey_service_amd.parallel.state import destroy_parallel, init_parallel
    st = init_parallel(tp=1, ep=2, device="cuda", backend="gloo")
    eng = _engine(model, st)
    eng.runner.keep_logits = True
    seqs = [eng.add_request(p, SamplingParams(max_tokens=4 if rank == 0 else 2)) for p in DPEP_PROMPTS[rank]]
    eng.step()
    eng.step()  # first decode step: routing fused into the norm, grouped skinny GEMMs, a2a
    logits = eng.runner.last_logits.float().cpu().clone()
    while eng.any_unfinished():
        eng.step()
    torch.save({"logits": logits, "tokens": [s.output_ids for s in seqs],
                "idle": eng.runner.stats.get("idle_steps", 0)}, f"{out_path}.{rank}")
    destroy_parallel()


def test_dp_attention_expert_all_to_all_on_gpu(tmp_path):
    """DP attention + EP=2 for the 8-expert Mixtral shape on the MI355X kernels (rank-sorted
    align / permute, grouped GEMMs over received rows, fused combine + add + RMSNorm): each
    rank's decode logits match a single-rank engine serving the same prompts."""
    from polykey_service_amd.engine import SamplingParams
    from polykey_service_amd.parallel.state import ParallelState
    model = "tiny-mixtral-e8"
    out = str(tmp_path / "dpep")
    mp.start_processes(_dpep_worker, args=(_port(), model, out), nprocs=2, join=True, start_method="spawn")
    ref = _engine(model, ParallelState(device=torch.device("cuda:0")))
    ref.runner.keep_logits = True
    for r in range(2):
        d = torch.load(f"{out}.{r}", weights_only=True)
        seqs = [ref.add_request(p, SamplingParams(max_tokens=4 if r == 0 else 2)) for p in DPEP_PROMPTS[r]]
        ref.step()
        ref.step()
        ref_logits = ref.runner.last_logits.float().cpu().clone()
        while ref.has_unfinished():
            ref.step()
        torch.testing.assert_close(d["logits"], ref_logits, atol=1e-1, rtol=5e-2)
        assert [t[0] for t in d["tokens"]] == [s.output_ids[0] for s in seqs]
    assert torch.load(f"{out}.1", weights_only=True)["idle"] > 0  # rank 1 served rank 0's rows after finishing
