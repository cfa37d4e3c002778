"""Decode-step time of the graph-captured engine (Llama-3-8B random init, 64 sequences, prompt
256), for A/B runs of kernel-library builds:

    python tools/ab_decode.py [--steps 128] [--reps 3]

decode ms/step = (T(prompt + 1 + steps new tokens) - T(1 new token)) / steps, best of ``reps``."""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from polykey_service_amd.engine.llm_engine import EngineConfig, LLMEngine  # noqa: E402
from polykey_service_amd.engine.sequence import SamplingParams  # noqa: E402


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="llama3-8b")
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--prompt", type=int, default=256)
    ap.add_argument("--steps", type=int, default=128)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--tag", default=os.environ.get("AB_TAG", ""))
    ap.add_argument("--eager", action="store_true", help="no HIP graphs (PMC runs count per dispatch)")
    a = ap.parse_args()
    max_len = max(2048, (a.prompt + a.steps + 64 + 511) // 512 * 512)
    eng = LLMEngine(EngineConfig(model=a.model, max_num_seqs=a.batch, device="cuda:0", max_model_len=max_len,
                                 hip_graphs=not a.eager))
    g = torch.Generator().manual_seed(0)
    hi = min(30000, eng.mcfg.vocab_size - 1)
    prompts = [torch.randint(10, hi, (a.prompt,), generator=g).tolist() for _ in range(a.batch)]

    def run(n: int) -> float:
        t0 = time.perf_counter()
        eng.generate(prompts, SamplingParams(max_tokens=n, ignore_eos=True, temperature=0.0))
        torch.cuda.synchronize()
        return time.perf_counter() - t0

    run(a.steps + 1)  # graphs captured, allocator warm
    per_step = []
    for _ in range(a.reps):
        full, one = run(a.steps + 1), run(1)
        per_step.append((full - one) / a.steps * 1e3)
    print(json.dumps({"tag": a.tag, "decode_ms_per_step": round(min(per_step), 4),
                      "all": [round(x, 4) for x in per_step], "batch": a.batch, "prompt": a.prompt}), flush=True)
    eng.shutdown()


if __name__ == "__main__":
    main()
