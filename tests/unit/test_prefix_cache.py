"""Automatic prefix caching: native block manager (csrc/runtime/block_manager.h) invariants and
engine-level equivalence (cached prefill == full prefill) on the CPU tiny model."""
import numpy as np
import pytest
import torch
from hypothesis import given, settings
from hypothesis import strategies as st

from polykey_service_amd._native.loader import load_extension
from polykey_service_amd.engine import EngineConfig, LLMEngine, SamplingParams
from polykey_service_amd.parallel.state import ParallelState

rt = load_extension("_pk_runtime")


def _toks(*vals):
    return np.asarray(vals, dtype=np.int32)


def test_prefix_hashes_chain():
    bm = rt.BlockManager(8, 4, 0, True)
    a = bm.prefix_hashes(_toks(1, 2, 3, 4, 5, 6, 7, 8, 9))
    b = bm.prefix_hashes(_toks(1, 2, 3, 4, 5, 6, 7, 0))
    c = bm.prefix_hashes(_toks(0, 2, 3, 4, 5, 6, 7, 8))
    assert len(a) == 2 and len(b) == 2  # full blocks only
    assert a[0] == b[0] and a[1] != b[1]  # same first block, different second
    assert c[0] != a[0] and c[1] != a[1]  # a different first block changes every later hash
    assert (a != 0).all()


def test_hash_key_and_salt():
    t = _toks(*range(8))
    a, b = rt.BlockManager(4, 4, 0, True), rt.BlockManager(4, 4, 0, True)
    assert (a.prefix_hashes(t) != b.prefix_hashes(t)).all()          # random per-process keys
    k1, k2 = rt.BlockManager(4, 4, 0, True, hash_key=7), rt.BlockManager(4, 4, 0, True, hash_key=7)
    assert (k1.prefix_hashes(t) == k2.prefix_hashes(t)).all()        # fixed key: reproducible
    assert (k1.prefix_hashes(t, salt=1) != k1.prefix_hashes(t, salt=2)).all()
    assert (k1.prefix_hashes(t, salt=0) == k1.prefix_hashes(t)).all()


def test_forged_hash_collision_is_not_served():
    """A lookup whose hashes equal a cached prefix's but whose tokens differ (a forged 64-bit
    collision) shares nothing; the mismatch is counted."""
    bm = rt.BlockManager(8, 4, 0, True)
    victim = _toks(*range(1, 9))
    h = bm.prefix_hashes(victim)
    assert bm.allocate(1, 8)
    bm.commit_prefix(1, h, victim, 2)
    attacker = _toks(1, 2, 3, 4, 99, 98, 97, 96)
    assert bm.match_prefix(2, h, attacker, 2) == 1       # only the genuinely equal first block
    assert bm.prefix_collisions == 1
    bm.free_seq(2)
    first_differs = _toks(0, 2, 3, 4, 5, 6, 7, 8)
    assert bm.match_prefix(3, h, first_differs, 2) == 0 and bm.prefix_collisions == 2
    # a block registered after a different parent is not reused under another parent's chain
    other = _toks(50, 51, 52, 53, 5, 6, 7, 8)
    h2 = bm.prefix_hashes(other)
    assert bm.allocate(5, 4)
    bm.commit_prefix(5, h2, other, 1)
    forged = np.array([h2[0], h[1]], dtype=np.uint64)   # block 1: equal tokens, other parent
    assert bm.match_prefix(4, forged, other, 2) == 1 and bm.prefix_collisions == 3


def test_match_commit_share_and_evict():
    bm = rt.BlockManager(6, 4, 0, True)
    toks = _toks(*range(1, 13))
    h = bm.prefix_hashes(toks)                           # 3 full blocks
    assert bm.match_prefix(1, h, toks, 3) == 0           # nothing cached yet
    assert bm.allocate(1, 12)
    bm.commit_prefix(1, h, toks, 2)                      # first 2 blocks computed
    assert bm.num_cached == 2
    t1 = bm.table(1)
    assert bm.match_prefix(2, h, toks, 3) == 2           # shares the committed blocks
    assert bm.table(2) == t1[:2] and bm.ref_count(t1[0]) == 2
    assert bm.allocate(2, 12) and bm.num_free == 6 - 3 - 1
    bm.free_seq(1)
    assert bm.ref_count(t1[0]) == 1 and bm.num_free == 6 - 3
    bm.free_seq(2)
    assert bm.num_free == 6 and bm.num_cached == 2       # cached blocks count as free
    assert bm.match_prefix(3, h, toks, 3) == 2           # still cached after release
    bm.free_seq(3)
    # exhausting the pool evicts the cached blocks (LRU) instead of failing
    assert bm.allocate(4, 24) and bm.num_free == 0 and bm.num_cached == 0
    bm.free_seq(4)
    assert bm.num_free == 6 and bm.match_prefix(5, h, toks, 3) == 0
    assert bm.prefix_hits == 4 and bm.prefix_queries == 12


def test_disabled_is_plain_allocator():
    bm = rt.BlockManager(4, 4, 0)
    t = _toks(*range(8))
    h = bm.prefix_hashes(t)
    assert bm.allocate(1, 8)
    bm.commit_prefix(1, h, t, 2)
    bm.free_seq(1)
    assert bm.num_cached == 0 and bm.match_prefix(2, h, t, 2) == 0 and bm.num_free == 4


def test_reset_prefix_cache():
    bm = rt.BlockManager(4, 2, 0, True)
    t = _toks(5, 6, 7, 8)
    h = bm.prefix_hashes(t)
    bm.allocate(1, 4)
    bm.commit_prefix(1, h, t, 2)
    bm.free_seq(1)
    assert bm.num_cached == 2
    bm.reset_prefix_cache()
    assert bm.num_cached == 0 and bm.num_free == 4 and bm.match_prefix(2, h, t, 2) == 0


@settings(max_examples=60, deadline=None)
@given(st.lists(st.tuples(st.sampled_from(["admit", "grow", "free"]), st.integers(0, 5), st.integers(1, 3)),
                max_size=60))
def test_refcounts_match_tables(ops):
    """Random admissions over 3 shared prefixes: every block's refcount equals the number of
    tables holding it, free + referenced = total, and freeing everything restores the pool."""
    bm = rt.BlockManager(24, 2, 0, True)
    ptoks = [_toks(*([p] * 8)) for p in range(3)]
    prefixes = [bm.prefix_hashes(t) for t in ptoks]
    live = {}
    for op, sid, arg in ops:
        if op == "admit" and sid not in live:
            h, t = prefixes[arg - 1], ptoks[arg - 1]
            bm.match_prefix(sid, h, t, 4)
            if bm.allocate(sid, 8):
                bm.commit_prefix(sid, h, t, 4)
                live[sid] = 8
            else:
                bm.free_seq(sid)
        elif op == "grow" and sid in live:
            if bm.allocate(sid, live[sid] + 2 * arg):
                live[sid] += 2 * arg
        elif op == "free" and sid in live:
            bm.free_seq(sid)
            del live[sid]
        refs = {}
        for s in live:
            for b in bm.table(s):
                refs[b] = refs.get(b, 0) + 1
        assert all(bm.ref_count(b) == n for b, n in refs.items())
        assert bm.num_free + len(refs) == 24
    for s in list(live):
        bm.free_seq(s)
    assert bm.num_free == 24 and bm.num_seqs == 0


def _engine(prefix_caching: bool) -> LLMEngine:
    return LLMEngine(EngineConfig(model="tiny-llama", max_num_seqs=8, max_num_batched_tokens=256, max_model_len=512,
                                  device="cpu", hip_graphs=False, prefix_caching=prefix_caching),
                     ParallelState(device=torch.device("cpu")))


def test_engine_cached_prefill_matches_full_prefill():
    torch.manual_seed(0)
    system = [1] + list(range(100, 170))           # shared 71-token "system prompt"
    first = system + [7, 8, 9]
    later = [system + [11, 12, 13, 14], system + list(range(300, 340)), system[:64] + [5, 6]]
    sp = SamplingParams(max_tokens=6, temperature=0.0, ignore_eos=True)
    ref = _engine(False)
    exp = ref.generate([first], sp) + ref.generate(later, sp)
    eng = _engine(True)
    got = eng.generate([first], sp)
    assert eng.scheduler.num_cached_tokens == 0
    got += eng.generate(later, sp)
    assert got == exp
    # 71 shared tokens = 2 full blocks of 32 for each later prompt (the third keeps 2 tokens to compute)
    assert eng.scheduler.num_cached_tokens == 3 * 64
    assert eng.bm.num_free == eng.bm.num_blocks and eng.bm.num_cached > 0


@pytest.mark.gpu
def test_engine_cached_prefill_matches_full_prefill_gpu():
    """Same equivalence on the MI355X kernels: the cached prompts run the paged-prefix prefill
    attention from a non-zero start, with HIP graphs for the decode steps."""
    def eng(pc):
        return LLMEngine(EngineConfig(model="tiny-llama-gqa4", max_num_seqs=8, max_num_batched_tokens=256,
                                      max_model_len=512, device="cuda:0", hip_graphs=True, prefix_caching=pc),
                         ParallelState(device=torch.device("cuda:0")))
    system = [1] + list(range(200, 300))
    first = system + [3, 4]
    later = [system + [9, 10, 11], system + list(range(400, 433))]
    sp = SamplingParams(max_tokens=5, temperature=0.0, ignore_eos=True)
    ref = eng(False)
    exp = ref.generate([first], sp) + ref.generate(later, sp)
    e = eng(True)
    got = e.generate([first], sp) + e.generate(later, sp)
    assert e.scheduler.num_cached_tokens == 2 * 96
    assert got == exp


def test_preempted_readmission_does_not_recount_cached_tokens():
    """A request whose prefix was a cache hit, preempted and re-admitted, re-matches its own
    committed blocks: usage.cached_tokens and the global count stay at the first admission's
    value and never exceed the prompt length."""
    from polykey_service_amd.engine.scheduler import Scheduler
    from polykey_service_amd.engine.sequence import Sequence
    bm = rt.BlockManager(32, 4, 0, True)
    sch = Scheduler(bm, max_num_seqs=4, max_num_batched_tokens=64, max_model_len=64)
    prompt = list(range(1, 14))                     # 13 tokens: 3 full blocks
    warm = Sequence("w", prompt, SamplingParams(max_tokens=4))
    sch.add(warm)
    b = sch.schedule()
    warm.num_computed += b.prefills[0][1]
    sch.commit_prefix(warm)
    seq = Sequence("s", prompt, SamplingParams(max_tokens=8))
    sch.add(seq)
    b = sch.schedule()
    assert seq.num_cached_tokens == 8 and sch.num_cached_tokens == 8  # 2 blocks (>= 2 tokens left)
    seq.num_computed += dict((s.request_id, n) for s, n in b.prefills)["s"]
    seq.output_ids += [5, 6, 7, 8]
    seq.num_computed += 3
    sch.commit_prefix(seq)
    assert sch._preempt_youngest(protect=warm) is seq
    b = sch.schedule()
    assert seq in [s for s, _ in b.prefills] and seq.num_computed > 0  # re-matched its own blocks
    assert seq.num_cached_tokens == 8 and sch.num_cached_tokens == 8
    assert seq.num_cached_tokens <= len(seq.prompt_ids)


def test_cache_salt_isolates_tenants():
    from polykey_service_amd.engine.scheduler import Scheduler
    from polykey_service_amd.engine.sequence import Sequence
    bm = rt.BlockManager(32, 4, 0, True)
    sch = Scheduler(bm, max_num_seqs=4, max_num_batched_tokens=64, max_model_len=64)
    prompt = list(range(1, 14))
    a = Sequence("a", prompt, SamplingParams(max_tokens=2, cache_salt="tenant-a"))
    sch.add(a)
    a.num_computed += sch.schedule().prefills[0][1]
    sch.commit_prefix(a)
    other = Sequence("b", prompt, SamplingParams(max_tokens=2, cache_salt="tenant-b"))
    same = Sequence("c", prompt, SamplingParams(max_tokens=2, cache_salt="tenant-a"))
    sch.add(other)
    sch.add(same)
    sch.schedule()
    assert other.num_cached_tokens == 0 and same.num_cached_tokens == 8
