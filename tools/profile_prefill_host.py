"""Host-side cost of the prefill steps at the start of a bench wave (64 x 256-token prompts after
a warm wave, HIP graphs on): cProfile of the two prefill engine steps -- the GPU idles while the
host builds the first step (tools/wave_gaps.py shows ~3 ms of gaps there)."""
import cProfile
import os
import pstats
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from polykey_service_amd.engine.llm_engine import EngineConfig, LLMEngine  # noqa: E402
from polykey_service_amd.engine.sequence import SamplingParams  # noqa: E402

model = sys.argv[1] if len(sys.argv) > 1 else "llama3-8b"
eng = LLMEngine(EngineConfig(model=model, device="cuda:0", max_num_seqs=64, max_model_len=1024, num_kv_blocks=4096,
                             overlap=True))
g = torch.Generator().manual_seed(0)


def wave(prof=None):
    for _ in range(64):
        eng.add_request(torch.randint(10, 30000, (256,), generator=g).tolist(),
                        SamplingParams(max_tokens=8, ignore_eos=True))
    steps = 0
    while eng.has_unfinished():
        if prof is not None and steps < 2:
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            prof.enable()
            eng.step()
            prof.disable()
            print(f"step {steps}: host {1e3 * (time.perf_counter() - t0):.2f} ms", flush=True)
        else:
            eng.step()
        steps += 1
    torch.cuda.synchronize()


wave()
wave()
pr = cProfile.Profile()
wave(pr)
pstats.Stats(pr).sort_stats("cumulative").print_stats(30)
