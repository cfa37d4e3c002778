"""Prefix caching on a shared system prompt (Llama-3-8B random init, one MI355X): a warm-up
request computes the shared prefix, then a wave of requests = shared prefix + unique suffix
runs with the cache on vs off.  Reports wave wall time, mean TTFT and the cached tokens.

    python tools/prefix_cache_bench.py [--batch 64] [--shared 1024] [--unique 64] [--out 32]
"""
import argparse
import json
import os
import random
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from polykey_service_amd.engine.llm_engine import EngineConfig, LLMEngine  # noqa: E402
from polykey_service_amd.engine.sequence import SamplingParams  # noqa: E402


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--shared", type=int, default=1024)
    ap.add_argument("--unique", type=int, default=64)
    ap.add_argument("--out", type=int, default=32)
    a = ap.parse_args()
    rng = random.Random(0)
    system = [rng.randrange(10, 30000) for _ in range(a.shared)]
    sp = SamplingParams(max_tokens=a.out, ignore_eos=True, temperature=0.0)
    for pc in (False, True):
        eng = LLMEngine(EngineConfig(model="llama3-8b", max_num_seqs=a.batch, device="cuda:0",
                                     max_model_len=4096, prefix_caching=pc))
        eng.generate([system + [5, 6, 7]], SamplingParams(max_tokens=2, ignore_eos=True))  # computes the prefix
        waves = []
        for w in range(2):
            prompts = [system + [rng.randrange(10, 30000) for _ in range(a.unique)] for _ in range(a.batch)]
            seqs = [eng.add_request(p, sp) for p in prompts]
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            while eng.has_unfinished():
                eng.step()
            torch.cuda.synchronize()
            wall = time.perf_counter() - t0
            ttft = sum(s.first_token_time - s.arrival for s in seqs) / len(seqs)
            waves.append((wall, ttft))
        wall, ttft = waves[-1]
        print(json.dumps({"prefix_caching": pc, "batch": a.batch, "shared": a.shared, "unique": a.unique,
                          "out": a.out, "wave_ms": round(wall * 1e3, 1), "mean_ttft_ms": round(ttft * 1e3, 1),
                          "cached_tokens_total": eng.scheduler.num_cached_tokens}), flush=True)
        del eng
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
