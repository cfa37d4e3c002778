"""TP=2 rehearsal of the Llama-3-8B decode path with both ranks on ONE MI355X: HIP-graph decode,
one-shot IPC all-reduce / all-gather, shared-memory step channel, pipelined continuations.
Start one process per rank (each may run under its own ``rocprofv3 --kernel-trace``):

    MASTER_ADDR=127.0.0.1 MASTER_PORT=29555 python tools/tp2_rehearsal.py --rank 0 --out r.json &
    MASTER_ADDR=127.0.0.1 MASTER_PORT=29555 python tools/tp2_rehearsal.py --rank 1 &

Rank 0 drives the engine (batch x prompt tokens, greedy, ignore_eos) and writes decode ms/step
plus the graph / continuation counters; rank 1 runs the worker loop.  With two ranks sharing
one GPU the step time is NOT a TP=2 number (both halves run on the same CUs); what the run
shows is the control plane: ``tools/tp2_gaps.py`` merges the two kernel traces and reports GPU
idle time per decode step (a per-step host sync on the worker would show as a gap per step)."""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--rank", type=int, required=True)
    ap.add_argument("--model", default="llama3-8b")
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--prompt", type=int, default=256)
    ap.add_argument("--steps", type=int, default=64)
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    os.environ.update(RANK=str(a.rank), WORLD_SIZE="2", LOCAL_RANK="0", POLYKEY_CUSTOM_AR="force")
    import torch

    from polykey_service_amd.engine import SamplingParams
    from polykey_service_amd.engine.llm_engine import EngineConfig, LLMEngine
    from polykey_service_amd.parallel.state import destroy_parallel, init_parallel

    st = init_parallel(tp=2, device="cuda", backend="gloo")
    assert st.custom_ar is not None, "custom all-reduce did not come up"
    blocks = a.batch * ((a.prompt + a.steps + 64) // 32 + 2) + 64
    eng = LLMEngine(EngineConfig(model=a.model, max_num_seqs=a.batch, max_model_len=1024, num_kv_blocks=blocks,
                                 hip_graphs=True, overlap=True, device="cuda:0"), st)
    if st.tp_rank != 0:
        eng.runner.worker_loop()
        print(json.dumps({"rank": 1, "worker_steps": eng.runner.stats.get("steps", 0)}), flush=True)
        destroy_parallel()
        return 0
    g = torch.Generator().manual_seed(0)
    hi = min(30000, eng.mcfg.vocab_size - 1)

    def run(n: int, salt: int) -> float:
        prompts = [[salt + 1] + torch.randint(10, hi, (a.prompt - 1,), generator=g).tolist() for _ in range(a.batch)]
        seqs = [eng.add_request(p, SamplingParams(max_tokens=n, ignore_eos=True, temperature=0.0)) for p in prompts]
        t0 = time.perf_counter()
        while eng.has_unfinished():
            eng.step()
        torch.cuda.synchronize()
        assert all(len(s.output_ids) == n for s in seqs)
        return time.perf_counter() - t0

    run(4, 0)  # warm-up (graphs already captured at init)
    t1 = run(1, 1)
    tn = run(1 + a.steps, 2)
    res = {"model": a.model, "tp": 2, "gpus": 1, "batch": a.batch, "prompt": a.prompt, "steps": a.steps,
           "decode_ms_per_step": round((tn - t1) / a.steps * 1e3, 3), "graph_steps": eng.runner.stats.get("graph_steps"),
           "continuations": eng.continuation_steps, "car_err": st.custom_ar.error()}
    eng.runner.stop_workers()
    print(json.dumps(res), flush=True)
    if a.out:
        with open(a.out, "w") as f:
            json.dump(res, f)
    destroy_parallel()
    return 0


if __name__ == "__main__":
    sys.exit(main())
