"""Prefill GEMM time against K at a fixed M x N (the 4-wave kernel and hipBLASLt): the intercept of
a linear fit is the per-tile fixed cost (prologue, epilogue stores, tail) that a persistent kernel
would overlap.   python tools/prefill_k_sweep.py [M] [N]"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from polykey_service_amd.ops import gemm_prefill  # noqa: E402


def t(fn, reps=8):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    b.synchronize()
    return a.elapsed_time(b) * 1e3 / reps


def main():
    M = int(sys.argv[1]) if len(sys.argv) > 1 else 8192
    N = int(sys.argv[2]) if len(sys.argv) > 2 else 28672
    rows = []
    for K in (1024, 2048, 4096, 8192, 16384):
        x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
        w = torch.randn(N, K, device="cuda", dtype=torch.bfloat16) * 0.02
        out = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
        ours = min(t(lambda: gemm_prefill.linear(x, w, out=out)) for _ in range(3))
        blas = min(t(lambda: torch.mm(x, w.t(), out=out)) for _ in range(3))
        rows.append((K, ours, blas))
        print(json.dumps({"M": M, "N": N, "K": K, "v6_us": round(ours, 1), "hipblaslt_us": round(blas, 1)}), flush=True)
    n = len(rows)
    for name, col in (("v6", 1), ("hipblaslt", 2)):
        mx = sum(r[0] for r in rows) / n
        my = sum(r[col] for r in rows) / n
        b = sum((r[0] - mx) * (r[col] - my) for r in rows) / sum((r[0] - mx) ** 2 for r in rows)
        print(json.dumps({"fit": name, "fixed_us": round(my - b * mx, 1), "us_per_k1024": round(b * 1024, 1)}))


if __name__ == "__main__":
    main()
