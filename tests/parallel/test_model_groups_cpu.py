"""Several models behind ONE front end on a one-process-per-GPU job, each on TP groups of its own
(``serve_models`` entries ``name@<gpus>[:tp<N>]``, adapters/local_llm.py
attach_model_groups).  Three gloo ranks on the CPU: tiny-llama-gqa4 at TP = 2 on ranks 0-1 (rank 0
is the front end and that group's leader) and tiny-llama at TP = 1 on rank 2 (its leader serves
its engine to rank 0 over the engine wire).  Every model's tokens over gRPC must be the tokens of
a single-process TP = 1 engine on the same seed, and stopping the front end releases every rank."""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

SPEC = "tiny-llama-gqa4@0-1:tp2,tiny-llama@2"
# the TP group away from rank 0: its leader is rank 1 (not dp_rank * tp_size)
SPEC2 = "tiny-llama@0,tiny-llama-gqa4@1-2:tp2"
PROMPTS = [[1, 5, 6, 7, 8, 9], [1] + list(range(20, 60)), [1, 2, 3], [1] + list(range(100, 130)),
           [1, 77, 78, 79], [1] + list(range(200, 212))]
MAXTOK = 5


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _cfg(spec=SPEC):
    from polykey_service_amd.config.server_config import ServerConfig
    return ServerConfig(backend="local", serve_models=spec, device="cpu", max_num_seqs=8, max_num_batched_tokens=128,
                        max_model_len=256, hip_graphs=False)


def _worker(rank, world, port, out, spec):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank), LOCAL_WORLD_SIZE=str(world), POLYKEY_PREFLIGHT="0",
                      POLYKEY_DIST_BACKEND="gloo")
    torch.set_num_threads(2)
    import grpc

    from polykey_service_amd import proto
    from polykey_service_amd.parallel.state import destroy_parallel
    from polykey_service_amd.server.app import build_service
    from polykey_service_amd.utils import slog
    from tests.helpers import ServerThread
    router = build_service(_cfg(spec), slog.Logger(open(os.devnull, "w")))
    if router is None:  # ranks 1 and 2: stopped by the front end
        destroy_parallel()
        return
    got = {}
    try:
        assert sorted(router.llm.llms) == ["tiny-llama", "tiny-llama-gqa4"]
        with ServerThread(router) as s, grpc.insecure_channel(s.addr) as ch:
            call = ch.unary_unary(proto.EXECUTE_TOOL, request_serializer=proto.ExecuteToolRequest.SerializeToString,
                                  response_deserializer=proto.ExecuteToolResponse.FromString)
            for model in ("tiny-llama", "tiny-llama-gqa4"):
                for i, p in enumerate(PROMPTS):
                    r = proto.ExecuteToolRequest(tool_name=f"llm.generate:{model}")
                    r.parameters.update({"prompt_token_ids": p, "max_tokens": MAXTOK, "ignore_eos": True,
                                         "temperature": 0.0, "return": "struct", "return_token_ids": True})
                    d = proto.struct_to_dict(call(r, timeout=120).struct_output)
                    assert d["model"] == model and d["usage"]["completion_tokens"] == MAXTOK, d
                    got[(model, i)] = [int(t) for t in d["token_ids"]]
    finally:
        router.llm.shutdown()
    torch.save(got, out)
    destroy_parallel()


@pytest.mark.parametrize("spec", [SPEC, SPEC2])
def test_two_models_on_tp_groups_behind_one_front_end(tmp_path, spec):
    from polykey_service_amd.adapters.local_llm import plan_model_groups
    from polykey_service_amd.engine import EngineConfig, LLMEngine, SamplingParams
    from polykey_service_amd.parallel.state import ParallelState
    assert plan_model_groups(SPEC, 3) == [("tiny-llama-gqa4", [0, 1]), ("tiny-llama", [2])]
    assert plan_model_groups(SPEC2, 3) == [("tiny-llama", [0]), ("tiny-llama-gqa4", [1, 2])]
    out = str(tmp_path / "fe.pt")
    mp.start_processes(_worker, args=(3, _port(), out, spec), nprocs=3, join=True, start_method="spawn")
    got = torch.load(out, weights_only=True)
    cfg = _cfg()
    compared = {}
    for model in ("tiny-llama", "tiny-llama-gqa4"):
        eng = LLMEngine(EngineConfig(model=model, max_num_seqs=8, max_num_batched_tokens=128, max_model_len=256,
                                     hip_graphs=False, device="cpu", seed=cfg.seed), ParallelState())
        eng.runner.keep_logits = True
        seqs = [eng.add_request(p, SamplingParams(max_tokens=MAXTOK, ignore_eos=True)) for p in PROMPTS]
        steps = []  # the reference's logits of every step (rows: the sequences in order)
        while eng.has_unfinished():
            eng.step()
            steps.append(eng.runner.last_logits.float())
        for i, s in enumerate(seqs):
            if model == "tiny-llama":  # TP = 1 in another process: identical
                assert got[(model, i)] == s.output_ids, (model, i, got[(model, i)], s.output_ids)
                continue
            # TP = 2: bf16 partials are rounded per rank, so the logits differ slightly; every token
            # must equal the reference's up to the first step whose top two logits are a near-tie
            # (after it the continuations may legitimately part ways)
            n = 0
            for t in range(MAXTOK):
                top2 = steps[t][i].topk(2).values
                if float(top2[0] - top2[1]) < 0.07:  # within 2 bf16 ulps at these logit magnitudes
                    break
                assert got[(model, i)][t] == s.output_ids[t], (model, i, t, got[(model, i)], s.output_ids)
                n += 1
            compared[(model, i)] = n
    # the comparison must not be vacuous: a third of the TP = 2 tokens, one whole sequence at least
    tp2 = [v for (m, _), v in compared.items() if m == "tiny-llama-gqa4"]
    assert sum(tp2) >= MAXTOK * len(PROMPTS) // 3 and max(tp2) == MAXTOK, compared


def test_plan_model_groups_validation():
    from polykey_service_amd.adapters.local_llm import parse_serve_models, parse_serve_plan, plan_model_groups
    assert parse_serve_plan("llama3-70b@0-3:tp4,llama3-8b@4,mixtral-8x7b@5-6") == [
        ("llama3-70b", [0, 1, 2, 3], 4), ("llama3-8b", [4], 1), ("mixtral-8x7b", [5, 6], 1)]
    assert plan_model_groups("llama3-70b@0-3:tp4,llama3-8b@4,mixtral-8x7b@5-6", 7) == [
        ("llama3-70b", [0, 1, 2, 3]), ("llama3-8b", [4]), ("mixtral-8x7b", [5]), ("mixtral-8x7b", [6])]
    # auto placement: tp devices from the free ones, in order
    assert plan_model_groups("a:tp2,b", 3) == [("a", [0, 1]), ("b", [2])]
    assert plan_model_groups("a@4-7:tp2,b@0-3:tp4", 8) == [("a", [4, 5]), ("a", [6, 7]), ("b", [0, 1, 2, 3])]
    with pytest.raises(ValueError, match="not a multiple"):
        parse_serve_plan("a@0-2:tp2")
    with pytest.raises(ValueError, match="covers ranks"):
        plan_model_groups("a@0-1:tp2", 3)  # rank 2 serves nothing
    with pytest.raises(ValueError, match="two models"):
        plan_model_groups("a@0-1,b@1", 2)
    with pytest.raises(ValueError, match="bad TP suffix"):
        parse_serve_plan("a@0:x2")
    with pytest.raises(ValueError, match="one process per GPU"):
        parse_serve_models("a@0-1:tp2")  # the single-process path serves TP = 1 only
