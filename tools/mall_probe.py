"""Probe: does a decode GEMM run faster when its weights were just read (Infinity Cache / MALL
warm) than when they are cold?  Decides whether prefetching the next projection's weights
during the latency-bound decode attention can pay.

For each shape, per iteration: read a buffer of the weight's size (either the GEMM's own
packed weight = "warm", or an unrelated buffer = "cold"), then time only the GEMM with events.
Weights rotate over > 1 GiB of copies so nothing else is cached.
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from polykey_service_amd.ops import gemm

gemm.SKINNY_ENABLED = True
M = 64
ws = torch.empty(16 * M * 131072, dtype=torch.float32, device="cuda")
x = None


def run(name, N, K, S, iters=30):
    global x
    x = torch.randn(M, K, device="cuda").to(torch.bfloat16)
    n = max(2, (1 << 30) // (N * K * 2) + 1)
    wl = [(torch.randn(N, K, device="cuda") * 0.02).to(torch.bfloat16) for _ in range(n)]
    pl = [gemm.pack_weight(w) for w in wl]
    other = [torch.empty_like(p) for p in pl[:2]]
    sink_b = torch.empty((), dtype=torch.bfloat16, device="cuda")

    def gemm_i(i):
        if S == 1:
            gemm.linear(x, wl[i], packed=pl[i])
        else:
            gemm.linear_partial(x, wl[i], ws, S, packed=pl[i])

    res = {}
    for mode in ("cold", "warm", "cold2", "warm2"):
        times = []
        for it in range(iters):
            i = it % n
            src = pl[i] if mode.startswith("warm") else other[it % 2]
            torch.amax(src.view(-1), 0, out=sink_b)  # one streaming read of the buffer
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            gemm_i(i)
            e.record()
            torch.cuda.synchronize()
            times.append(s.elapsed_time(e) * 1000.0)
        times.sort()
        res[mode] = times[len(times) // 2]
    print(f"{name:8s} N={N:6d} K={K:5d} S={S:2d} MiB={N*K*2/2**20:6.1f} | " +
          " ".join(f"{k} {v:6.2f}us" for k, v in res.items()), flush=True)
    del wl, pl, other
    torch.cuda.empty_cache()


for name, N, K, S in [("qkv", 6144, 4096, 4), ("o", 4096, 4096, 8), ("down", 4096, 14336, 8),
                      ("gate_up", 28672, 4096, 1)]:
    run(name, N, K, S)
