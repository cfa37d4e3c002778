"""DP single front end on the MI355X: two engine ranks (sharing the one GPU of the test box, so
gloo carries the rank handshake) behind ONE gRPC front end on rank 0 (engine/remote.py
dp_gateway), driven through bench.py --frontend single with HIP graphs on."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def test_single_front_end_two_engine_ranks():
    args = ["--gpus", "2", "--frontend", "single", "--model", "tiny-llama-gqa4", "--steps", "1", "--warmup", "1",
            "--concurrency", "8", "--prompt-len", "32", "--max-tokens", "16", "--num-kv-blocks", "1024",
            "--tp-extra-model", "none"]
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py")] + args, cwd=REPO, capture_output=True,
                       text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    out = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][0])
    assert out["config"]["parallelism"] == "dp2_single_frontend" and out["config"]["global_batch"] == 16
    assert out["config"]["hip_graphs"] is True
    # every request of both replicas completed through the one front end
    assert out["value"] == pytest.approx(16 * 16 / (out["ms_per_step"] / 1000.0), rel=0.02)
