"""Tensor-parallel rehearsal at a model's REAL per-rank shapes with every rank on ONE MI355X.

An 8-GPU node is not always available, but 8 shards of Llama-3-70B (17.6 GB each, block-packed
only) fit in one MI355X's 288 GB, so the whole TP=8 decode path can run at its real widths:
H 8192, one KV head per rank (GQA 8 in the fused decode attention), 16,128-row padded LM-head
shards, W=8 one-shot / fused IPC collectives, HIP graphs, the shared-memory step channel and
pipelined continuations.  Step times are NOT TP=8 numbers (all ranks share one GPU's CUs and
HBM); what a run proves is correctness at shape and the control plane (kernel traces).

    python tools/tp_rehearsal.py --world 8 --model llama3-70b [--layers 8] [--ref run] [--prof]

Roles (the launcher starts the others as child processes, no exec):
  ref   TP = 1 engine on the same seed (packed-only weights for 70B), eager: first-step logits
        of the comparison prompts and their greedy tokens -> <out>/ref.pt
  rank  one TP rank; rank 0 drives: (1) eager greedy tokens (graphs set aside), (2) the same
        prompts through the HIP graphs with continuations, (3) a timed decode run; writes
        <out>/result.json with eager == graph, the comparison with ref.pt and the counters.
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

CMP_PROMPTS = [[1, 5, 6, 7, 8, 9], [1] + list(range(20, 60)), [1, 2], [1] + list(range(300, 557))]
# TP = N prefill logits may differ from TP = 1 by at most this many times the TP = 1 rounding
# noise at the same depth (_noise); a dropped rank partial lands far outside (tests/parallel/
# test_tp8_shapes_gpu.py injects one)
NOISE_FACTOR = 3.0


def _port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _engine(a, st, graphs: bool, device: str):
    from polykey_service_amd.engine.llm_engine import EngineConfig, LLMEngine
    blocks = a.batch * ((a.prompt + a.steps + 96) // 32 + 2) + 256
    return LLMEngine(EngineConfig(model=a.model, num_layers=a.layers, max_num_seqs=max(a.batch, len(CMP_PROMPTS)),
                                  max_num_batched_tokens=a.max_batched, max_model_len=1024, num_kv_blocks=blocks,
                                  hip_graphs=graphs, overlap=graphs, graph_batch_sizes=(len(CMP_PROMPTS), a.batch),
                                  device=device, prefix_caching=False), st)
    # prefix caching off: the comparison runs repeat the same prompts, and a prefill over a cached
    # prefix rounds differently from a full one (bf16 logits of random weights have exact ties)


def _greedy(eng, prompts, n, keep_first=False):
    import torch
    from polykey_service_amd.engine import SamplingParams
    eng.runner.keep_logits = keep_first
    seqs = [eng.add_request(list(p), SamplingParams(max_tokens=n, ignore_eos=True, temperature=0.0)) for p in prompts]
    eng.step()
    first = eng.runner.last_logits.float().cpu().clone() if keep_first else None
    eng.runner.keep_logits = False
    while eng.has_unfinished():
        eng.step()
    torch.cuda.synchronize()
    return [list(s.output_ids) for s in seqs], first


def role_ref(a) -> int:
    import torch
    from polykey_service_amd.parallel.state import ParallelState
    t0 = time.perf_counter()
    eng = _engine(a, ParallelState(device=torch.device("cuda:0")), graphs=False, device="cuda:0")
    init_s = time.perf_counter() - t0
    toks, first = _greedy(eng, CMP_PROMPTS, a.cmp_tokens, keep_first=True)
    noise = _noise(eng, a)
    torch.save({"tokens": toks, "logits": first, "init_s": init_s,
                "noise_mean": [p["mean_abs_diff"] for p in noise["prompts"]],
                "noise_max": [p["max_abs_diff"] for p in noise["prompts"]]}, os.path.join(a.out, "ref.pt"))
    with open(os.path.join(a.out, "noise.json"), "w") as f:
        json.dump(noise, f, indent=1)
    print(json.dumps({"role": "ref", "init_s": round(init_s, 1), "tokens0": [t[:4] for t in toks], "noise": noise}),
          flush=True)
    return 0


def _noise(eng, a) -> dict:
    """Calibration for the TP = N vs TP = 1 logits comparison: how far apart two equally valid
    TP = 1 computations of the same prefill land at this depth (random weights amplify bf16
    rounding-order noise layer by layer).  Each comparison prompt alone: its prefill in one step
    vs in two halves (the second over the first's cached KV: other GEMM tiles, attention over a
    cached prefix), the logits of its last token compared."""
    import torch
    from polykey_service_amd.engine import SamplingParams
    out = {"layers": eng.mcfg.num_layers, "prompts": []}
    sch = eng.scheduler
    saved = (sch.max_num_batched_tokens, getattr(sch, "max_prefill_chunk", None))
    for p in CMP_PROMPTS:
        lg = []
        for budget in (a.max_batched, (len(p) + 1) // 2):
            sch.max_num_batched_tokens = budget
            sch.max_prefill_chunk = budget
            eng.runner.keep_logits = True
            eng.add_request(list(p), SamplingParams(max_tokens=1, ignore_eos=True, temperature=0.0))
            while eng.has_unfinished():
                eng.step()  # the last step completes the prompt and samples from its logits
            torch.cuda.synchronize()
            lg.append(eng.runner.last_logits.float().cpu()[-1].clone())
        d = (lg[0] - lg[1]).abs()
        out["prompts"].append({"len": len(p), "max_abs_diff": round(float(d.max()), 4),
                               "mean_abs_diff": round(float(d.mean()), 5), "scale": round(float(lg[0].abs().mean()), 4),
                               "argmax_equal": int(lg[0].argmax()) == int(lg[1].argmax()),
                               "top2_gap": round(float(lg[0].topk(2).values[0] - lg[0].topk(2).values[1]), 4)})
    sch.max_num_batched_tokens, sch.max_prefill_chunk = saved[0], saved[1]
    eng.runner.keep_logits = False
    return out


def role_noise(a) -> int:
    import torch
    from polykey_service_amd.parallel.state import ParallelState
    eng = _engine(a, ParallelState(device=torch.device("cuda:0")), graphs=False, device="cuda:0")
    out = _noise(eng, a)
    print(json.dumps(out), flush=True)
    with open(os.path.join(a.out, "noise.json"), "w") as f:
        json.dump(out, f, indent=1)
    return 0


def _near_tie_ok(got, ref, logits, tie=0.15):
    """Greedy first tokens equal, or the TP token is a near-tie of the reference's argmax."""
    bad = []
    for row, (g, r) in enumerate(zip(got, ref)):
        if g[0] != r[0]:
            lg = logits[row]
            if float(lg[g[0]]) < float(lg.max()) - tie:
                bad.append(row)
    return bad


def _steps_logits(eng, prompts, n):
    import torch
    from polykey_service_amd.engine import SamplingParams
    seqs = [eng.add_request(list(p), SamplingParams(max_tokens=n, ignore_eos=True, temperature=0.0)) for p in prompts]
    out = []
    while eng.has_unfinished():
        eng.step()
        torch.cuda.synchronize()
        out.append(eng.runner.last_logits.float().cpu().clone())
    return out, [list(s.output_ids) for s in seqs]


def _debug_compare(eng, a):
    """Eager vs graphed, step by step: max |diff| of the logits and each row's top-2 gap."""
    graphs, short = eng.runner.graphs, eng.runner.short_graphs
    eng.runner.graphs, eng.runner.short_graphs = {}, {}
    le, te = _steps_logits(eng, CMP_PROMPTS, a.cmp_tokens)
    eng.runner.graphs, eng.runner.short_graphs = graphs, short
    lg, tg = _steps_logits(eng, CMP_PROMPTS, a.cmp_tokens)
    rows = []
    for k, (x, y) in enumerate(zip(le, lg)):
        n = min(x.shape[0], y.shape[0])
        d = (x[:n] - y[:n]).abs()
        top = x[:n].topk(2, -1).values
        rows.append({"step": k, "max_abs_diff": round(float(d.max()), 5),
                     "row_max_diff": [round(float(v), 4) for v in d.max(-1).values],
                     "top2_gap": [round(float(v), 4) for v in (top[:, 0] - top[:, 1])]})
    return {"steps": rows, "tokens_equal": te == tg}


def role_rank(a) -> int:
    import torch
    from polykey_service_amd.parallel.state import destroy_parallel, init_parallel
    st = init_parallel(tp=a.world, device="cuda", backend="gloo")
    assert st.custom_ar is not None, "custom all-reduce did not come up"
    t0 = time.perf_counter()
    eng = _engine(a, st, graphs=True, device="cuda:0")
    init_s = time.perf_counter() - t0
    if st.tp_rank != 0:
        eng.runner.worker_loop()
        destroy_parallel()
        return 0
    print(json.dumps({"phase": "rank0 engine ready", "init_s": round(init_s, 1)}), flush=True)
    res = {"model": a.model, "layers": eng.mcfg.num_layers, "tp": a.world, "gpus": 1, "init_s": round(init_s, 1),
           "vocab_local": eng.model.vocab_local, "lm_head_packed": eng.model.lm_head_p is not None,
           "packed_only": bool(getattr(eng.model, "packed_only", False)),
           "graph_buckets": sorted(eng.runner.graphs)}
    # (1) eager: graphs set aside, so leader and workers run every kernel eagerly
    graphs, short = eng.runner.graphs, eng.runner.short_graphs
    eng.runner.graphs, eng.runner.short_graphs = {}, {}
    eager, first = _greedy(eng, CMP_PROMPTS, a.cmp_tokens, keep_first=True)
    eng.runner.graphs, eng.runner.short_graphs = graphs, short
    if a.check_only:  # the reference comparison only (fault-injection runs)
        graphed = graphed_nc = None
    # (2) the same prompts through the decode graphs, with pipelined continuations
    else:
        eng.overlap = False  # graphs, one scheduled step at a time (no continuations)
        if eng.runner.debug_logits:  # step-by-step logits, eager vs graphed
            res["debug"] = _debug_compare(eng, a)
        graphed_nc, _ = _greedy(eng, CMP_PROMPTS, a.cmp_tokens)
        eng.overlap = True
        g0, c0 = eng.runner.stats["graph_steps"], eng.continuation_steps
        graphed, _ = _greedy(eng, CMP_PROMPTS, a.cmp_tokens)
        res.update(graph_equals_eager=graphed == eager, graph_no_continuation_equals_eager=graphed_nc == eager,
                   graph_steps=eng.runner.stats["graph_steps"] - g0,
                   continuations=eng.continuation_steps - c0, tokens0=[t[:6] for t in eager],
                   graph_tokens0=[t[:6] for t in graphed], graph_nc_tokens0=[t[:6] for t in graphed_nc])
    ref_path = os.path.join(a.out, "ref.pt")
    if os.path.exists(ref_path):
        ref = torch.load(ref_path, weights_only=True)
        rl = ref["logits"]
        diff = (first - rl).abs()
        row_mean = [round(float(v), 5) for v in diff.mean(-1)]
        res.update(ref_first_tokens_equal=[t[0] for t in eager] == [t[0] for t in ref["tokens"]],
                   ref_first_token_rows_not_near_tie=_near_tie_ok(eager, ref["tokens"], rl),
                   ref_logits_max_abs_diff=round(float(diff.max()), 4),
                   ref_logits_mean_abs_diff=round(float(diff.mean()), 5),
                   ref_logits_row_mean_abs_diff=row_mean,
                   ref_logits_scale=round(float(rl.abs().mean()), 4),
                   ref_tokens_equal_all=eager == ref["tokens"])
        if "noise_mean" in ref:
            # every comparison prompt: TP = N vs TP = 1 within NOISE_FACTOR x the TP = 1 noise at this
            # depth (the largest over the prompts: a prompt whose two TP = 1 computations happen to
            # be bit-identical -- row-independent decode GEMMs for <= 64-token steps -- says nothing
            # about the scale of a valid reordering)
            nm = ref["noise_mean"]
            band = NOISE_FACTOR * max(nm)
            res.update(ref_noise_row_mean_abs_diff=nm, ref_noise_band=round(band, 5),
                       ref_rows_outside_noise=[r for r, d in enumerate(row_mean) if d > band])
    if a.check_only:
        eng.runner.stop_workers()
        print(json.dumps(res), flush=True)
        with open(os.path.join(a.out, "result.json"), "w") as f:
            json.dump(res, f, indent=1)
        destroy_parallel()
        return 0
    # (3) timed decode: batch x prompt, 1 token vs 1 + steps tokens
    g = torch.Generator().manual_seed(0)
    hi = min(30000, eng.mcfg.vocab_size - 1)

    def run(n: int, salt: int) -> float:
        prompts = [[salt + 1] + torch.randint(10, hi, (a.prompt - 1,), generator=g).tolist() for _ in range(a.batch)]
        t = time.perf_counter()
        _greedy(eng, prompts, n)
        return time.perf_counter() - t
    run(2, 0)
    t1 = run(1, 1)
    tn = run(1 + a.steps, 2)
    res.update(batch=a.batch, prompt=a.prompt, steps=a.steps,
               decode_ms_per_step_shared_gpu=round((tn - t1) / a.steps * 1e3, 3),
               car_err=st.custom_ar.error(), tp_push_calls=getattr(eng.model, "_push_calls", 0),
               fused_tp_decode=eng.model._rowscale_ok(
                   torch.zeros((a.batch, eng.mcfg.hidden_size), dtype=torch.bfloat16, device="cuda:0")))
    eng.runner.stop_workers()
    print(json.dumps(res), flush=True)
    with open(os.path.join(a.out, "result.json"), "w") as f:
        json.dump(res, f, indent=1)
    destroy_parallel()
    return 0


def launch(a) -> int:
    os.makedirs(a.out, exist_ok=True)
    me = [sys.executable, os.path.abspath(__file__)]
    common = ["--world", str(a.world), "--model", a.model, "--layers", str(a.layers), "--batch", str(a.batch),
              "--prompt", str(a.prompt), "--steps", str(a.steps), "--out", a.out, "--cmp-tokens", str(a.cmp_tokens),
              "--max-batched", str(a.max_batched)] + (["--check-only"] if a.check_only else []) + (
              ["--force-overlap"] if a.force_overlap else [])
    env = dict(os.environ, PYTHONPATH=ROOT + os.pathsep + os.environ.get("PYTHONPATH", ""))
    if a.ref == "run":
        print(json.dumps({"phase": "ref"}), flush=True)
        r = subprocess.run(me + common + ["--role", "ref"], env=env, timeout=a.timeout)
        if r.returncode != 0:
            print(json.dumps({"error": "reference run failed", "rc": r.returncode}), flush=True)
            return 1
    port = _port()
    procs = []
    for r in range(a.world):
        e = dict(env, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(r), WORLD_SIZE=str(a.world),
                 LOCAL_RANK="0", LOCAL_WORLD_SIZE=str(a.world), POLYKEY_CUSTOM_AR="force",
                 POLYKEY_CUSTOM_AR_TIMEOUT_S=os.environ.get("POLYKEY_CUSTOM_AR_TIMEOUT_S", "120"))
        if a.hw_queues:
            e["GPU_MAX_HW_QUEUES"] = str(a.hw_queues)
        cmd = me + common + ["--role", "rank", "--rank", str(r)]
        if a.prof:
            cmd = ["rocprofv3", "--kernel-trace", "--output-format", "csv", "-d", os.path.join(a.out, f"trace_r{r}"),
                   "--"] + cmd
        log = open(os.path.join(a.out, f"rank{r}.log"), "w")
        procs.append((subprocess.Popen(cmd, env=e, stdout=log, stderr=subprocess.STDOUT), log))
    deadline = time.monotonic() + a.timeout
    t_start = time.monotonic()

    def heartbeat():  # a long init (80 layers x 8 ranks) must not look like a hang to a supervisor
        while any(p.poll() is None for p, _ in procs):
            time.sleep(20)
            print(json.dumps({"elapsed_s": round(time.monotonic() - t_start), "alive": sum(p.poll() is None for p, _ in procs)}),
                  flush=True)
    import threading
    threading.Thread(target=heartbeat, daemon=True).start()
    rcs = []
    for p, log in procs:
        try:
            rcs.append(p.wait(timeout=max(1.0, deadline - time.monotonic())))
        except subprocess.TimeoutExpired:
            for q, _ in procs:
                q.kill()
            rcs.append(-9)
        log.close()
    print(json.dumps({"rank_exit_codes": rcs}), flush=True)
    return 0 if all(rc == 0 for rc in rcs) else 1


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--role", choices=["launch", "ref", "rank", "noise"], default="launch")
    ap.add_argument("--rank", type=int, default=0)
    ap.add_argument("--world", type=int, default=8)
    ap.add_argument("--model", default="llama3-70b")
    ap.add_argument("--layers", type=int, default=0, help="0: the preset's depth")
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--prompt", type=int, default=256)
    ap.add_argument("--steps", type=int, default=32)
    ap.add_argument("--cmp-tokens", type=int, default=8)
    ap.add_argument("--max-batched", type=int, default=8192)
    ap.add_argument("--ref", choices=["none", "run", "file"], default="none")
    ap.add_argument("--prof", action="store_true", help="each rank under rocprofv3 --kernel-trace")
    ap.add_argument("--check-only", action="store_true",
                    help="rank 0: the eager reference comparison only (no graph runs, no timed decode)")
    ap.add_argument("--timeout", type=float, default=1000.0)
    # one HW queue per rank: 8 processes x the default 4 queues oversubscribe the hardware scheduler,
    # which then time-slices the ranks and every collective waits for a slice (4-layer 70B TP=8
    # rehearsal: 7.4 ms / step at 1 queue per rank, 128 ms at 2, ~500 ms at the default)
    ap.add_argument("--hw-queues", type=int, default=1, help="GPU_MAX_HW_QUEUES per rank (0: the box default)")
    ap.add_argument("--force-overlap", action="store_true",
                    help="take the chunked comm-stream TP chain (POLYKEY_TP_DECODE_CHUNKS) although the ranks share "
                         "one GPU (models/llama.py force_overlap_streams)")
    ap.add_argument("--out", default=os.path.join(ROOT, "gpurun_out", "tp_rehearsal"))
    a = ap.parse_args()
    if a.role == "ref":
        return role_ref(a)
    if a.role == "noise":
        os.makedirs(a.out, exist_ok=True)
        return role_noise(a)
    if a.force_overlap:
        from polykey_service_amd.models.llama import LlamaForCausalLM
        LlamaForCausalLM.force_overlap_streams = True
    if a.role == "rank":
        return role_rank(a)
    return launch(a)


if __name__ == "__main__":
    sys.exit(main())
