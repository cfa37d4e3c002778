"""Backend choice of parallel/state.py: RCCL for one rank per GPU, gloo otherwise."""
import pytest

from polykey_service_amd.parallel.state import init_parallel, pick_backend


@pytest.mark.parametrize("dev,n_dev,local,override,exp", [
    ("cuda", 8, 8, None, "nccl"),     # one rank per GPU on an 8-GPU node
    ("cuda", 1, 1, None, "nccl"),
    ("cuda", 1, 2, None, "gloo"),     # rehearsing 2 ranks on a one-GPU box
    ("cuda", 8, 16, None, "gloo"),
    ("cpu", 0, 2, None, "gloo"),
    ("cuda", 1, 2, "nccl", "nccl"),   # POLYKEY_DIST_BACKEND / explicit argument wins
    ("cuda", 8, 8, "gloo", "gloo"),
])
def test_pick_backend(dev, n_dev, local, override, exp):
    assert pick_backend(dev, n_dev, local, override) == exp


def test_single_process_state(monkeypatch):
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    st = init_parallel(device="cpu")
    assert (st.world_size, st.tp_size, st.dp_size, st.rank) == (1, 1, 1, 0)
    with pytest.raises(ValueError):
        monkeypatch.setenv("WORLD_SIZE", "3")
        init_parallel(tp=2, device="cpu")
