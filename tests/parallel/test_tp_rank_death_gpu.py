"""The dead-rank contract on the GPU path (2 ranks on one MI355X: IPC collectives, HIP graphs,
step channel): SIGKILL one rank mid-decode and the survivor exits non-zero within the bound --
the front end via the IPC collective's timeout (sticky error word) and NOT_SERVING, a worker via
its leader's vanished pid (tests/rank_death.py)."""
import pytest

from tests.rank_death import run_kill

pytestmark = pytest.mark.gpu
NOT_SERVING = 2


@pytest.mark.timeout(600)
def test_worker_death_ends_the_front_end_gpu(tmp_path):
    rc, dt, seen, got, logs = run_kill(tmp_path, "tiny-llama-gqa4", gpu=True, victim=1, bound_s=90)
    assert rc is not None and rc != 0, f"front end still running {dt:.1f}s after the worker died\n{logs}"
    assert NOT_SERVING in seen, (seen, logs)


@pytest.mark.timeout(600)
def test_leader_death_ends_the_worker_gpu(tmp_path):
    rc, dt, seen, got, logs = run_kill(tmp_path, "tiny-llama-gqa4", gpu=True, victim=0, bound_s=90)
    assert rc is not None and rc != 0, f"worker still running {dt:.1f}s after the leader died\n{logs}"
