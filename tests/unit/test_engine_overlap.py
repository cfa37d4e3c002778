"""Pipelined engine steps (EngineConfig.overlap): same tokens as the synchronous loop, aborts
while a step is in flight are dropped, and every request finishes."""
import torch

from polykey_service_amd.engine import EngineConfig, LLMEngine, SamplingParams
from polykey_service_amd.parallel.state import ParallelState


def _engine(overlap: bool) -> LLMEngine:
    return LLMEngine(EngineConfig(model="tiny-llama", max_num_seqs=8, max_num_batched_tokens=64, max_model_len=256,
                                  device="cpu", hip_graphs=False, overlap=overlap),
                     ParallelState(device=torch.device("cpu")))


def test_overlap_matches_sync_generate():
    prompts = [[1, 5, 6, 7], [1] + list(range(20, 60)), [1, 9]]
    sp = SamplingParams(max_tokens=7, temperature=0.8, seed=11)
    a = _engine(False).generate(prompts, sp)
    b = _engine(True).generate(prompts, sp)
    assert a == b and all(len(x) == 7 for x in a)


def test_overlap_outputs_lag_one_step_and_abort_in_flight():
    e = _engine(True)
    s1 = e.add_request([1, 2, 3], SamplingParams(max_tokens=5, ignore_eos=True), "r1")
    e.add_request([1, 4, 5], SamplingParams(max_tokens=5, ignore_eos=True), "r2")
    assert e.step() == []            # first batch launched, nothing completed yet
    outs = e.step()                  # completes the prefill step
    assert sorted(o.request_id for o in outs) == ["r1", "r2"]
    e.abort("r2")                    # r2 is part of the batch in flight
    seen = []
    while e.has_unfinished():
        seen += e.step()
    assert all(o.request_id == "r1" for o in seen)
    assert len(s1.output_ids) == 5 and seen[-1].finished
    assert e.bm.num_free == e.bm.num_blocks


def test_before_schedule_admits_arrivals_into_the_next_step():
    """A request that arrives while a step is in flight (AsyncLLM's queue, drained by the
    before_schedule hook) joins the step scheduled right after that one completes."""
    e = _engine(True)
    e.add_request([1, 2, 3], SamplingParams(max_tokens=3, ignore_eos=True), "r1")
    sizes = []
    orig = e.scheduler.schedule

    def schedule():
        b = orig()
        sizes.append(sorted(s.request_id for s, _ in b.prefills))
        return b
    e.scheduler.schedule = schedule
    assert e.step() == []            # r1's prefill in flight
    arrivals = [("r2", [1, 4, 5])]

    def drain():
        while arrivals:
            rid, p = arrivals.pop()
            e.add_request(p, SamplingParams(max_tokens=3, ignore_eos=True), rid)
    e.before_schedule = drain
    e.step()
    assert sizes[:2] == [["r1"], ["r2"]], sizes
    while e.has_unfinished():
        e.step()
    assert e.bm.num_free == e.bm.num_blocks


def test_abort_in_before_schedule_drops_the_completed_output():
    e = _engine(True)
    e.add_request([1, 2, 3], SamplingParams(max_tokens=4, ignore_eos=True), "r1")
    e.add_request([1, 4, 5], SamplingParams(max_tokens=4, ignore_eos=True), "r2")
    assert e.step() == []
    fired = []

    def drain():
        if not fired:
            fired.append(e.abort("r2"))
    e.before_schedule = drain
    outs = e.step()
    assert [o.request_id for o in outs] == ["r1"], outs
    seen = []
    while e.has_unfinished():
        seen += e.step()
    assert all(o.request_id == "r1" for o in seen) and seen[-1].finished
    assert e.bm.num_free == e.bm.num_blocks
