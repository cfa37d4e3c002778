"""Host-side cost of one engine step (64 decoding sequences, HIP graphs): cProfile of the
engine loop plus a wall-clock breakdown, to size the CPU work between GPU steps."""
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
eng = LLMEngine(EngineConfig(model=model, device="cuda:0", max_num_seqs=64, max_model_len=2048, num_kv_blocks=4096,
                             overlap=True))
g = torch.Generator().manual_seed(0)
for _ in range(64):
    eng.add_request(torch.randint(10, 1000, (256,), generator=g).tolist(),
                    SamplingParams(max_tokens=1000, ignore_eos=True))
for _ in range(20):
    eng.step()
torch.cuda.synchronize()
n = 100
t0 = time.perf_counter()
pr = cProfile.Profile()
pr.enable()
for _ in range(n):
    eng.step()
pr.disable()
torch.cuda.synchronize()
dt = (time.perf_counter() - t0) / n
print(f"step wall {dt * 1e3:.2f} ms")
pstats.Stats(pr).sort_stats("tottime").print_stats(25)
