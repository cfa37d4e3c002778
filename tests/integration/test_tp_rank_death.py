"""A TP rank that dies mid-decode ends the whole group (CPU, gloo, 2 server processes): the
survivor exits non-zero within the bound -- the front end after flipping health to NOT_SERVING,
a worker as soon as its leader's process is gone -- so the supervisor restarts the group instead
of it hanging forever (tests/rank_death.py)."""
import pytest

from tests.rank_death import run_kill

NOT_SERVING = 2


@pytest.mark.timeout(300)
def test_worker_death_ends_the_front_end(tmp_path):
    rc, dt, seen, got, logs = run_kill(tmp_path, "tiny-llama-gqa4", gpu=False, victim=1, bound_s=60)
    assert rc is not None and rc != 0, f"front end still running {dt:.1f}s after the worker died\n{logs}"
    assert NOT_SERVING in seen, (seen, logs)
    assert got["error"] is not None, "the in-flight stream did not fail"


@pytest.mark.timeout(300)
def test_leader_death_ends_the_worker(tmp_path):
    rc, dt, seen, got, logs = run_kill(tmp_path, "tiny-llama-gqa4", gpu=False, victim=0, bound_s=60)
    assert rc is not None and rc != 0, f"worker still running {dt:.1f}s after the leader died\n{logs}"
    assert dt < 30, dt
