"""bench.py driver contract on the CPU (tiny random-init model, gloo for 2 ranks): one JSON line
from rank 0 with the BASELINE metric, whole-job value, and the DP parallelism / global batch
of the launch; 2 ranks go through the torchrun child launch the driver itself uses."""
import json
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
def _run(cmd, cwd, env, timeout=300):
    """bench.py in its own session: on a timeout the whole tree (torchrun, its ranks, load
    generators) is killed, not just the launcher."""
    p = subprocess.Popen(cmd, cwd=cwd, env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True,
                         start_new_session=True)
    try:
        out, err = p.communicate(timeout=timeout)
    except subprocess.TimeoutExpired:
        sys.path.insert(0, REPO)
        from bench import kill_tree
        kill_tree(p)
        try:
            out, err = p.communicate(timeout=30)
        except subprocess.TimeoutExpired:
            out, err = "", ""
        pytest.fail(f"bench.py timed out after {timeout} s\n{err[-3000:]}")
    return subprocess.CompletedProcess(cmd, p.returncode, out, err)


ARGS = ["--model", "tiny-llama-gqa4", "--steps", "1", "--warmup", "1", "--concurrency", "4", "--prompt-len", "8",
        "--max-tokens", "4", "--no-graphs"]


@pytest.mark.parametrize("gpus,client,frontend", [(1, "process", "replicas"), (2, "process", "replicas"),
                                                 (1, "inproc", "replicas"), (3, "inproc", "single"),
                                                 (2, "inproc", "single")])
def test_bench_json_line(tmp_path, gpus, client, frontend):
    env = dict(os.environ, CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="")
    r = _run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", str(gpus), "--client", client,
              "--frontend", frontend] + ARGS, tmp_path, env)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout
    out = json.loads(lines[0])
    assert out["metric"].startswith("output tokens/sec via gRPC")
    assert out["n_gpus"] == gpus and out["steps"] == 1 and out["warmup"] == 1
    assert out["value"] > 0 and out["ms_per_step"] > 0 and out["higher_is_better"] is True
    assert out["scaling"] == "weak" and out["dtype"] == "bf16"
    gw = {"single": "_single_frontend"}.get(frontend, "") if gpus > 1 else ""
    assert not any(k.startswith("tp") for k in out)  # no TP child for a model other than Llama-3-8B
    assert out["config"]["parallelism"] == f"dp{gpus}{gw}" and out["config"]["global_batch"] == 4 * gpus
    assert out["config"]["clients"] == ("load-generator process" if client == "process" else "server event loop")
    # unique random prompts: the prefix cache serves nothing, so no prefill work is skipped
    assert out["config"]["prefix_caching"] is True and out["config"]["prefix_cache_hit_tokens"] == 0
    # every request completed its 4 tokens: tokens / elapsed over ranks = value
    assert out["value"] == pytest.approx(4 * 4 * gpus / (out["ms_per_step"] / 1000.0), rel=0.02)


def test_bench_openai_chat_route():
    """VERDICT r5 item 8 / BASELINE config 4's route: --mode openai drives POST /v1/chat/completions
    (api/openai.py on the server's process) with templated prompts of exactly --prompt-len tokens;
    the same JSON contract, the route named in config.rpc."""
    env = dict(os.environ, CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="")
    r = _run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "1", "--mode", "openai"] + ARGS[:-1]
             + ["--prompt-len", "160", "--no-graphs"], REPO, env)
    assert r.returncode == 0, r.stderr[-2000:]
    out = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][0])
    assert out["config"]["rpc"].startswith("POST /v1/chat/completions") and out["config"]["seq_len"] == 160
    assert out["config"]["prefix_cache_hit_tokens"] == 0
    assert out["value"] == pytest.approx(4 * 4 / (out["ms_per_step"] / 1000.0), rel=0.02)


def test_bench_dp_attention_expert_all_to_all():
    """Mixtral-shaped MoE with DP attention + EP=2 (expert all-to-all between the two ranks'
    engines, lockstep steps, coordinated shutdown) through the same torchrun child launch."""
    env = dict(os.environ, CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="")
    args = ["--model", "tiny-mixtral", "--ep", "2", "--steps", "1", "--warmup", "1", "--concurrency", "3",
            "--prompt-len", "8", "--max-tokens", "4", "--no-graphs"]
    r = _run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2"] + args, REPO, env)
    assert r.returncode == 0, r.stderr[-2000:]
    out = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][0])
    assert out["config"]["parallelism"] == "dp2_ep2_a2a" and out["config"]["global_batch"] == 6
    assert out["value"] == pytest.approx(3 * 4 * 2 / (out["ms_per_step"] / 1000.0), rel=0.02)


def test_bench_world8_reports_tp_child():
    """The 8-GPU driver launch (torchrun, 8 ranks running bench.py --gpus 8) on the CPU: rank 0
    relays the replica measurement of a fresh 8-rank child and adds the TP=8 child's result under
    tp8_<model> (a 70B-shaped tiny model: 8 kv heads, GQA 8, ragged vocab); a TP child that fails
    leaves the replica number intact."""
    env = dict(os.environ, CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="", OMP_NUM_THREADS="1")
    base = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=8",
            "--master-addr", "127.0.0.1", "--master-port", "0", os.path.join(REPO, "bench.py"), "--gpus", "8",
            "--model", "tiny-llama-g8", "--steps", "1", "--warmup", "1", "--concurrency", "2", "--prompt-len", "128",
            "--max-tokens", "3", "--no-graphs"]  # (128: the TP child's chat template alone is 100 byte tokens)
    r = _run(base + ["--tp-extra-model", "tiny-llama-g8", "--ep-extra-model", "tiny-mixtral-e8"], REPO, env,
             timeout=900)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout
    out = json.loads(lines[0])
    assert out["n_gpus"] == 8 and out["config"]["parallelism"] == "dp8" and out["config"]["global_batch"] == 16
    assert out["value"] == pytest.approx(2 * 3 * 8 / (out["ms_per_step"] / 1000.0), rel=0.02)
    tp = out["tp8_tiny-llama-g8"]
    assert "error" not in tp, tp
    assert tp["parallelism"] == "tp8" and tp["global_batch"] == 2 and tp["scaling"] == "strong"
    assert tp["rpc"].startswith("POST /v1/chat/completions"), tp  # config 4: the OpenAI chat route
    assert tp["value"] == pytest.approx(2 * 3 / (tp["ms_per_step"] / 1000.0), rel=0.02)
    # BASELINE config 5 -- an 8-expert MoE with DP attention + EP = 8 (expert
    # all-to-all over the 8 ranks) under ep8_<model>, 2 clients per replica
    ep = out["ep8_tiny-mixtral-e8"]
    assert "error" not in ep, ep
    assert ep["parallelism"] == "dp8_ep8_a2a" and ep["global_batch"] == 16 and ep["scaling"] == "weak", ep
    assert ep["value"] == pytest.approx(2 * 3 * 8 / (ep["ms_per_step"] / 1000.0), rel=0.02)
    # a TP child that cannot run (unknown model) is reported in its key, the main number stays
    r = _run(base + ["--tp-extra-model", "no-such-model", "--tp-extra-timeout", "120", "--ep-extra-model",
                     "no-such-moe", "--ep-extra-timeout", "120"], REPO, env, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    out = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][0])
    assert out["value"] > 0 and "error" in out["tp8_no-such-model"] and "error" in out["ep8_no-such-moe"]


def test_bench_world8_hung_tp_child_meets_the_deadline():
    """a TP child that hangs (test hook) is killed inside the ONE --deadline,
    and the main JSON line -- the replica number plus the TP key's error -- is printed before it."""
    import time
    env = dict(os.environ, CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="", OMP_NUM_THREADS="1",
               POLYKEY_TEST_HOOKS="1", POLYKEY_BENCH_HANG="tp")
    deadline = 150
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=8", "--master-addr",
           "127.0.0.1", "--master-port", "0", os.path.join(REPO, "bench.py"), "--gpus", "8", "--model",
           "tiny-llama-g8", "--steps", "1", "--warmup", "1", "--concurrency", "2", "--prompt-len", "8",
           "--max-tokens", "3", "--no-graphs", "--tp-extra-model", "tiny-llama-g8", "--deadline", str(deadline)]
    t0 = time.monotonic()
    r = _run(cmd, REPO, env, timeout=deadline + 120)
    wall = time.monotonic() - t0
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout
    out = json.loads(lines[0])
    assert out["value"] > 0 and out["config"]["parallelism"] == "dp8"
    assert "timeout" in out["tp8_tiny-llama-g8"]["error"], out["tp8_tiny-llama-g8"]
    assert wall < deadline + 30, wall  # torchrun's own teardown aside, the line came within the deadline
