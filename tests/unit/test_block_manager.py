"""Native BlockManager (csrc/runtime/block_manager.cpp): allocation invariants + step packing."""
import numpy as np
import pytest
from hypothesis import given, settings
from hypothesis import strategies as st

from polykey_service_amd._native.loader import load_extension

rt = load_extension("_pk_runtime")


def test_alloc_free_roundtrip():
    bm = rt.BlockManager(10, 16, 1)
    assert bm.num_free == 10 and bm.blocks_for(17) == 2
    assert bm.allocate(1, 33) and bm.num_free == 7 and len(bm.table(1)) == 3
    assert bm.allocate(1, 40) and bm.num_free == 7  # still 3 blocks
    assert not bm.allocate(2, 16 * 8)  # needs 8 > 7 free
    assert bm.num_free == 7 and not bm.has(2)
    assert bm.can_allocate(2, 16 * 6, True) and not bm.can_allocate(2, 16 * 7, True)  # watermark 1
    bm.free_seq(1)
    assert bm.num_free == 10 and bm.num_seqs == 0


@settings(max_examples=60, deadline=None)
@given(st.lists(st.tuples(st.integers(0, 5), st.integers(0, 200), st.booleans()), max_size=60))
def test_no_leaks_or_double_allocation(ops):
    bm = rt.BlockManager(32, 8, 0)
    live = {}
    for sid, toks, free in ops:
        if free:
            bm.free_seq(sid)
            live.pop(sid, None)
        elif bm.allocate(sid, toks):
            live[sid] = max(live.get(sid, 0), bm.blocks_for(toks))
        tables = [bm.table(s) for s in live]
        used = [b for t in tables for b in t]
        assert len(used) == len(set(used)), "block owned twice"
        assert bm.num_free + len(used) == 32
        for s in live:
            assert len(bm.table(s)) >= live[s]


def test_pack_step():
    bm = rt.BlockManager(16, 4, 0)
    assert bm.allocate(7, 6) and bm.allocate(9, 3)
    sids = np.array([9, 7], dtype=np.int64)
    ncomp = np.array([2, 0], dtype=np.int32)
    nnew = np.array([1, 6], dtype=np.int32)
    toks = np.array([100, 1, 2, 3, 4, 5, 6], dtype=np.int32)
    ids, pos, slots = (np.zeros(16, np.int32) for _ in range(3))
    bt = np.full((4, 8), -1, np.int32)
    cl = np.zeros(4, np.int32)
    cu = np.zeros(5, np.int32)
    T = bm.pack_step(sids, ncomp, nnew, toks, ids, pos, slots, bt, 8, cl, cu)
    assert T == 7
    assert list(ids[:7]) == [100, 1, 2, 3, 4, 5, 6] and list(pos[:7]) == [2, 0, 1, 2, 3, 4, 5]
    t9, t7 = bm.table(9), bm.table(7)
    assert slots[0] == t9[0] * 4 + 2
    assert list(slots[1:7]) == [t7[p // 4] * 4 + p % 4 for p in range(6)]
    assert list(cl[:2]) == [3, 6] and list(cu[:3]) == [0, 1, 7]
    assert list(bt[1, :2]) == t7 and bt[1, 2] == 0
    with pytest.raises(RuntimeError):
        bm.pack_step(np.array([42], np.int64), ncomp[:1], nnew[:1], toks, ids, pos, slots, bt, 8, cl, cu)
