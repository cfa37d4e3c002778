"""Prefill GEMMs (Llama-3-8B, 8192 tokens) on hipBLASLt: weight layout [N, K] (F.linear, the
engine's layout) vs [K, N] (x @ W^T stored transposed), cold weights.  TF/s per shape."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import torch.nn.functional as F

T = int(sys.argv[1]) if len(sys.argv) > 1 else 8192
shapes = [("qkv", 6144, 4096), ("o", 4096, 4096), ("gate_up", 28672, 4096), ("down", 4096, 14336)]


def timeit(fn, n, iters=20):
    for i in range(3):
        fn(i % n)
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for i in range(iters):
        fn(i % n)
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1000.0


tot = {"nk": 0.0, "kn": 0.0}
for name, N, K in shapes:
    x = torch.randn(T, K, device="cuda").to(torch.bfloat16)
    n = max(2, (1 << 29) // (N * K * 2) + 1)
    w_nk = [(torch.randn(N, K, device="cuda") * 0.02).to(torch.bfloat16) for _ in range(n)]
    out = torch.empty(T, N, device="cuda", dtype=torch.bfloat16)
    t_nk = timeit(lambda i: torch.matmul(x, w_nk[i].t(), out=out), n)
    w_kn = [w.t().contiguous() for w in w_nk]
    del w_nk
    t_kn = timeit(lambda i: torch.matmul(x, w_kn[i], out=out), n)
    del w_kn
    fl = 2.0 * T * N * K
    tot["nk"] += t_nk
    tot["kn"] += t_kn
    print(f"{name:8s} T={T} N={N:6d} K={K:5d} | [N,K] {t_nk:8.1f}us {fl / t_nk / 1e6:7.1f} TF/s | "
          f"[K,N] {t_kn:8.1f}us {fl / t_kn / 1e6:7.1f} TF/s", flush=True)
    torch.cuda.empty_cache()
print(f"layer total: [N,K] {tot['nk']:.1f}us  [K,N] {tot['kn']:.1f}us", flush=True)
