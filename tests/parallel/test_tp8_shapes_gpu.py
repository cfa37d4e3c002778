"""Llama-3-70B TP=8 at its REAL per-rank shapes, 8 ranks on one MI355X:
hidden 8192, one KV head per rank (GQA 8 in the fused decode attention), 16,128-row padded
LM-head shards on the packed decode GEMM, W=8 one-shot / fused IPC collectives, HIP graphs,
pipelined continuations, the shared-memory step channel; 4 of the 80 layers (the full depth runs
in tools/tp_rehearsal.py).  The graphed engine must emit exactly the eager engine's tokens, and
its prefill logits must match a TP=1 engine on the same seed to within 3x the TP=1 engine's own
rounding noise at this depth (the same prefill in one step vs in two halves, the largest over the
comparison prompts).  A
deliberately wrong model -- one rank's attention partial dropped in one layer -- must fail that
check."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def _rehearse(out, extra=(), env=None):
    cmd = [sys.executable, os.path.join(ROOT, "tools", "tp_rehearsal.py"), "--world", "8", "--model", "llama3-70b",
           "--layers", "4", "--batch", "16", "--prompt", "64", "--steps", "8", "--cmp-tokens", "6", "--ref", "run",
           "--max-batched", "1024", "--timeout", "420", "--out", out] + list(extra)
    r = subprocess.run(cmd, timeout=480, capture_output=True, text=True, env=env)
    logs = "".join(open(os.path.join(out, f)).read()[-3000:] for f in sorted(os.listdir(out)) if f.endswith(".log"))
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:] + logs
    res = json.load(open(os.path.join(out, "result.json")))
    print(json.dumps(res))
    return res


def test_llama3_70b_tp8_shapes_on_one_gpu(tmp_path):
    res = _rehearse(str(tmp_path / "tp8"))
    assert res["layers"] == 4 and res["tp"] == 8
    assert res["vocab_local"] == 16128 and res["lm_head_packed"], res
    assert res["fused_tp_decode"], ("decode did not take the fused TP collective chain", json.dumps(res))
    assert res["car_err"] == 0
    assert res["graph_steps"] > 0 and res["continuations"] > 0, res
    assert res["graph_equals_eager"], res
    assert res["ref_first_token_rows_not_near_tie"] == [], res
    # bf16 partials are rounded per rank before the sum: logits agree to the TP=1 noise, not bits
    assert res["ref_noise_band"] > 0, res  # the calibration measured something
    assert res["ref_rows_outside_noise"] == [], res


def test_llama3_70b_tp8_overlapped_collectives(tmp_path):
    """The TP decode chain with every row-parallel collective overlapped with its GEMM (column-chunk
    GEMMs, chunk collectives forked to the comm stream inside the captured graph), forced on for the
    shared-GPU rehearsal with the box's default hardware queues: graphs equal eager, logits inside
    the TP=1 noise band."""
    env = dict(os.environ, POLYKEY_TP_DECODE_CHUNKS="2")
    res = _rehearse(str(tmp_path / "tp8o"), ["--hw-queues", "0", "--force-overlap"], env=env)
    assert res["fused_tp_decode"] and res["car_err"] == 0 and res["graph_steps"] > 0, res
    assert res["graph_equals_eager"] and res["ref_rows_outside_noise"] == [], res


def test_llama3_70b_tp8_pushed_collectives(tmp_path):
    """The row-parallel projections' GEMM epilogues push their tiles into the owner ranks' slots
    (POLYKEY_TP_PUSH, gemm.push_projection + custom_ar.reduce_residual_pushed): graphs equal eager,
    logits inside the TP=1 noise band, and the decode steps really took the pushed path."""
    env = dict(os.environ, POLYKEY_TP_PUSH="1")
    res = _rehearse(str(tmp_path / "tp8p"), env=env)
    assert res["fused_tp_decode"] and res["car_err"] == 0 and res["graph_steps"] > 0, res
    assert res["tp_push_calls"] > 0, res
    assert res["graph_equals_eager"] and res["ref_rows_outside_noise"] == [], res


def test_llama3_70b_tp8_dropped_partial_is_caught(tmp_path):
    """Fault injection: rank 3 drops its attention partial in layer 1 (POLYKEY_FAULT_DROP_PARTIAL);
    every comparison prompt's logits must leave the noise band."""
    env = dict(os.environ, POLYKEY_FAULT_DROP_PARTIAL="1,3", POLYKEY_TEST_HOOKS="1")
    res = _rehearse(str(tmp_path / "tp8f"), ["--check-only"], env=env)
    assert res["ref_noise_band"] > 0 and len(res["ref_rows_outside_noise"]) == 4, res
