"""Sequence-parallel shard layout (parallel/comm.py SPLayout) — index logic only, no process
group: every padded row belongs to exactly one rank's shard, chunk by chunk, in the order the
per-chunk reduce-scatter / all-gather calls of sp_reduce_scatter / sp_all_gather produce."""
from unittest import mock

from hypothesis import given, settings
from hypothesis import strategies as st

from polykey_service_amd.parallel import comm
from polykey_service_amd.parallel.state import ParallelState


def _layout(T, tp, rank, chunks):
    with mock.patch.object(comm, "get_state", lambda: ParallelState(world_size=tp, tp_size=tp, tp_rank=rank)):
        return comm.SPLayout(T, chunks)


@settings(max_examples=60, deadline=None)
@given(T=st.integers(1, 3000), tp=st.sampled_from([1, 2, 4, 8]), chunks=st.sampled_from([1, 2, 3, 4]))
def test_shards_partition_padded_rows(T, tp, chunks):
    owner = {}
    for r in range(tp):
        lay = _layout(T, tp, r, chunks)
        assert lay.Tp >= T and lay.Tp % (tp * chunks) == 0 and lay.Tp - T < tp * chunks
        assert lay.rows * tp == lay.Tp
        seen = 0
        for c in range(chunks):
            lo, hi, slo, shi = lay.chunk(c)
            assert hi - lo == tp * (shi - slo)
            assert slo == seen  # a rank's pieces are contiguous in its shard, chunk-major
            seen = shi
            for j in range(shi - slo):
                row = lo + r * (shi - slo) + j  # all_gather_into_tensor puts rank r's piece r-th
                assert row not in owner
                owner[row] = (r, slo + j)
        assert seen == lay.rows
    assert sorted(owner) == list(range(_layout(T, tp, 0, chunks).Tp))


def test_overlap_chunks_grow_with_the_prefill():
    """Prefill collectives overlap with up to 4 row chunks, each of >= OVERLAP_MIN_ROWS rows."""
    from polykey_service_amd.parallel import comm
    m = comm.OVERLAP_MIN_ROWS
    assert comm.overlap_chunks(m) == 1 and comm.overlap_chunks(2 * m - 1) == 1
    assert comm.overlap_chunks(2 * m) == 2 and comm.overlap_chunks(4 * m - 1) == 2
    assert comm.overlap_chunks(4 * m) == 4 and comm.overlap_chunks(64 * m) == 4
