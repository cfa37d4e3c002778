"""Scheduler policy: budgets, chunked prefill, FIFO admission, preemption (CPU, no model)."""
import pytest
from hypothesis import given, settings
from hypothesis import strategies as st

from polykey_service_amd._native.loader import load_extension
from polykey_service_amd.engine.scheduler import Scheduler
from polykey_service_amd.engine.sequence import FinishReason, SamplingParams, Sequence, SeqStatus

rt = load_extension("_pk_runtime")


def mk(n_prompt, max_tokens=4):
    return Sequence(f"r{n_prompt}-{id(object())}", list(range(1, n_prompt + 1)), SamplingParams(max_tokens=max_tokens))


def simulate_step(sched, batch, tok=7):
    sampling = batch.sampling_seqs()
    for s, n in batch.prefills:
        s.num_computed += n
    for s in batch.decodes:
        s.num_computed += 1
    for s in sampling:
        r = s.append_token(tok, 0.0)
        if r:
            sched.finish(s, r)
    sched.remove_finished()


def test_budget_and_chunking():
    bm = rt.BlockManager(1000, 16, 0)
    sch = Scheduler(bm, max_num_seqs=4, max_num_batched_tokens=100, max_model_len=1024)
    a, b = mk(70), mk(70)
    sch.add(a)
    sch.add(b)
    bt = sch.schedule()
    assert [(s is a, n) for s, n in bt.prefills] == [(True, 70), (False, 30)]
    assert bt.sampling_seqs() == [a]
    simulate_step(sch, bt)
    bt2 = sch.schedule()
    assert bt2.decodes == [a] and [(s is b, n) for s, n in bt2.prefills] == [(True, 40)]


def test_max_num_seqs():
    bm = rt.BlockManager(1000, 16, 0)
    sch = Scheduler(bm, max_num_seqs=2, max_num_batched_tokens=1000, max_model_len=1024)
    for _ in range(3):
        sch.add(mk(5))
    bt = sch.schedule()
    assert len(bt.prefills) == 2 and len(sch.waiting) == 1


def test_preempts_youngest_and_recovers():
    bm = rt.BlockManager(4, 4, 0)  # 16 tokens of KV in total
    sch = Scheduler(bm, max_num_seqs=4, max_num_batched_tokens=64, max_model_len=64)
    a, b = mk(7, max_tokens=6), mk(7, max_tokens=6)
    sch.add(a)
    sch.add(b)
    finished = []
    for _ in range(60):
        if not sch.has_work():
            break
        bt = sch.schedule()
        done_before = {s.request_id for s in (a, b) if s.is_finished()}
        simulate_step(sch, bt)
        finished += [s for s in (a, b) if s.is_finished() and s.request_id not in done_before]
    assert a.is_finished() and b.is_finished()
    assert sch.num_preemptions >= 1 and b.num_preemptions >= 1 and a.num_preemptions == 0
    assert len(a.output_ids) == 6 and len(b.output_ids) == 6
    assert bm.num_free == 4


def test_abort_frees_blocks():
    bm = rt.BlockManager(100, 16, 0)
    sch = Scheduler(bm, 8, 256, 1024)
    s = mk(40)
    sch.add(s)
    sch.schedule()
    assert bm.num_free < 100
    assert sch.abort(s.request_id) is s and s.finish_reason == FinishReason.ABORT
    assert bm.num_free == 100 and not sch.has_work()


def test_too_long_prompt_rejected_and_max_tokens_clamped():
    bm = rt.BlockManager(100, 16, 0)
    sch = Scheduler(bm, 8, 256, 64)
    with pytest.raises(ValueError):
        sch.add(mk(64))
    s = mk(60, max_tokens=100)
    sch.add(s)
    assert s.params.max_tokens == 4


@settings(max_examples=40, deadline=None)
@given(st.lists(st.tuples(st.integers(1, 60), st.integers(1, 12)), min_size=1, max_size=12),
       st.integers(3, 40), st.integers(8, 64))
def test_everything_finishes_without_leaks(reqs, blocks, budget):
    bm = rt.BlockManager(blocks, 8, 0)
    sch = Scheduler(bm, 6, budget, 512)
    seqs = []
    for p, m in reqs:
        s = mk(p, m)
        try:
            sch.add(s)
            seqs.append(s)
        except ValueError:
            pass
    for _ in range(5000):
        if not sch.has_work():
            break
        bt = sch.schedule()
        assert bt.num_tokens <= budget
        simulate_step(sch, bt)
    assert not sch.has_work()
    for s in seqs:
        assert len(s.output_ids) == s.params.max_tokens
    assert bm.num_free == blocks


def test_prefill_first_wave_and_decode_stall_cap():
    """prefill_first: a wave of 4 prompts of 100 tokens (budget 200) admitted while 2 sequences
    decode runs as two whole 200-token prefill steps; the decodes wait at most
    max_decode_stall steps.  decode_first mixes the decodes in and leaves a tail chunk."""
    def run(policy, stall=4):
        bm = rt.BlockManager(1000, 16, 0)
        sch = Scheduler(bm, max_num_seqs=8, max_num_batched_tokens=200, max_model_len=1024, policy=policy,
                        max_decode_stall=stall)
        old = [mk(10, 50), mk(10, 50)]
        for s in old:
            sch.add(s)
        simulate_step(sch, sch.schedule())
        for _ in range(4):
            sch.add(mk(100, 5))
        steps = []
        for _ in range(3):
            b = sch.schedule()
            steps.append((len(b.decodes), [n for _, n in b.prefills]))
            simulate_step(sch, b)
        return steps
    assert run("prefill_first") == [(0, [100, 100]), (0, [100, 100]), (6, [])]
    assert run("prefill_first", stall=1) == [(0, [100, 100]), (4, [100, 96]), (5, [4])]
    assert run("decode_first") == [(2, [100, 98]), (3, [2, 100, 95]), (5, [5])]
    with pytest.raises(ValueError):
        Scheduler(rt.BlockManager(10, 16, 0), policy="fastest")


def test_younger_sequence_never_evicts_an_older_one():
    """Two sequences that cannot both hold their KV (5 + 5 blocks of 9): the younger one must
    yield to the older, or under prefill-first they preempt each other forever."""
    reqs = [(51, 4), (46, 5), (50, 8), (33, 10), (30, 9), (41, 5), (18, 4), (2, 2), (40, 12)]
    bm = rt.BlockManager(9, 8, 0)
    sch = Scheduler(bm, 6, 19, 512)
    seqs = []
    for p, m in reqs:
        s = mk(p, m)
        sch.add(s)
        seqs.append(s)
    for _ in range(2000):
        if not sch.has_work():
            break
        simulate_step(sch, sch.schedule())
    assert not sch.has_work() and all(s.is_finished() for s in seqs)
    assert bm.num_free == 9
