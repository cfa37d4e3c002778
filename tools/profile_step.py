"""Engine-level profiling driver: Llama-3-8B (random init) serving 64 concurrent requests
(prompt 256, 64 new tokens) through LLMEngine, eager (no HIP graphs) so every kernel dispatch
is visible to ``rocprofv3 --kernel-trace`` / ``--pmc``.

    cd /tmp && export TMPDIR=/tmp
    rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE FETCH_SIZE \\
        --output-format csv -d $REPO/gpurun_out/pmc -- python3 $REPO/tools/profile_step.py
"""
import argparse
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
    ap.add_argument("--max-tokens", type=int, default=64)
    ap.add_argument("--graphs", action="store_true")
    a = ap.parse_args()
    eng = LLMEngine(EngineConfig(model=a.model, hip_graphs=a.graphs, max_num_seqs=max(64, a.batch), device="cuda:0",
                                 max_model_len=4096, num_kv_blocks=8192))
    g = torch.Generator().manual_seed(0)
    hi = min(30000, eng.mcfg.vocab_size - 1)
    prompts = [torch.randint(10, hi, (a.prompt,), generator=g).tolist() for _ in range(a.batch)]
    sp = SamplingParams(max_tokens=a.max_tokens, ignore_eos=True, temperature=0.0)
    t0 = time.perf_counter()
    out = eng.generate(prompts, sp)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    n = sum(len(o) for o in out)
    print(f"profile_step: {n} tokens in {dt:.2f}s ({n / dt:.0f} tok/s incl. prefill)", flush=True)
    eng.shutdown()


if __name__ == "__main__":
    main()
