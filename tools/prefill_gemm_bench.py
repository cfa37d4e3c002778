"""Prefill GEMM shapes on hipBLASLt: F.linear vs matmul(out=), and torch._grouped_mm for MoE.

Times each call with CUDA events (median of 20 after 5 warmup) on random bf16 data and
prints TF/s.  Shapes: Llama-3-8B prefill at 8192 rows (QKV / O / gate_up / down) and the
Mixtral expert GEMMs at ~4096 rows per expert.

    python tools/prefill_gemm_bench.py
"""
import json
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))
from polykey_service_amd.ops import gemm_prefill  # noqa: E402


def timeit(fn, reps=20, warm=5):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        b.synchronize()
        ts.append(a.elapsed_time(b) * 1e3)
    ts.sort()
    return ts[len(ts) // 2]


def main():
    dev = "cuda"
    torch.manual_seed(0)
    rows = []
    for name, M, N, K in [("qkv", 8192, 6144, 4096), ("o", 8192, 4096, 4096), ("gate_up", 8192, 28672, 4096),
                          ("down", 8192, 4096, 14336), ("o4k", 4096, 4096, 4096), ("o16k", 16384, 4096, 4096)]:
        x = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
        w = torch.randn(N, K, device=dev, dtype=torch.bfloat16) * 0.02
        out = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        fl = 2.0 * M * N * K
        t1 = timeit(lambda: F.linear(x, w))
        t2 = timeit(lambda: torch.matmul(x, w.t(), out=out))
        t3 = timeit(lambda: torch.mm(x, w.t(), out=out))
        rows.append({"gemm": name, "M": M, "N": N, "K": K, "linear_us": round(t1, 1), "linear_tfs": round(fl / t1 / 1e6, 1),
                     "matmul_out_us": round(t2, 1), "matmul_out_tfs": round(fl / t2 / 1e6, 1),
                     "mm_out_us": round(t3, 1)})
        for v in (4,):
            tv = timeit(lambda: gemm_prefill.linear(x, w, out=out, variant=v))
            rows[-1][f"pk{v}_us"] = round(tv, 1)
            rows[-1][f"pk{v}_tfs"] = round(fl / tv / 1e6, 1)
        print(json.dumps(rows[-1]), flush=True)
    # Mixtral experts: 8 experts, 32768 routed rows (16384 tokens x top-2), uneven split
    E, H, I = 8, 4096, 14336
    counts = [4096 + d for d in (512, -256, 128, -384, 0, 256, -128, -128)]
    T = sum(counts)
    offs = torch.tensor([0] + list(torch.tensor(counts).cumsum(0)), dtype=torch.int32, device=dev)
    x = torch.randn(T, H, device=dev, dtype=torch.bfloat16)
    w13 = torch.randn(E, 2 * I, H, device=dev, dtype=torch.bfloat16) * 0.02
    h = torch.randn(T, I, device=dev, dtype=torch.bfloat16)
    w2 = torch.randn(E, H, I, device=dev, dtype=torch.bfloat16) * 0.02
    fl13 = 2.0 * T * 2 * I * H
    fl2 = 2.0 * T * H * I

    def loop13():
        lo = 0
        for e, c in enumerate(counts):
            F.linear(x[lo:lo + c], w13[e])
            lo += c

    def loop2():
        lo = 0
        for e, c in enumerate(counts):
            F.linear(h[lo:lo + c], w2[e])
            lo += c
    r = {"gemm": "moe_loop", "w13_us": round(timeit(loop13, 5, 2), 1), "w2_us": round(timeit(loop2, 5, 2), 1)}
    r["w13_tfs"] = round(fl13 / r["w13_us"] / 1e6, 1)
    r["w2_tfs"] = round(fl2 / r["w2_us"] / 1e6, 1)
    print(json.dumps(r), flush=True)
    for v in (4,):
        g13 = timeit(lambda: gemm_prefill.grouped_linear(x, w13, offs, silu=True, variant=v), 5, 2)
        g2 = timeit(lambda: gemm_prefill.grouped_linear(h, w2, offs, variant=v), 5, 2)
        print(json.dumps({"gemm": f"pk_grouped{v}", "w13_silu_us": round(g13, 1), "w13_tfs": round(fl13 / g13 / 1e6, 1),
                          "w2_us": round(g2, 1), "w2_tfs": round(fl2 / g2 / 1e6, 1)}), flush=True)
    try:
        o32 = offs[1:].contiguous()
        g13 = timeit(lambda: torch._grouped_mm(x, w13.transpose(1, 2), offs=o32), 5, 2)
        g2 = timeit(lambda: torch._grouped_mm(h, w2.transpose(1, 2), offs=o32), 5, 2)
        print(json.dumps({"gemm": "torch._grouped_mm", "w13_us": round(g13, 1), "w13_tfs": round(fl13 / g13 / 1e6, 1),
                          "w2_us": round(g2, 1), "w2_tfs": round(fl2 / g2 / 1e6, 1)}), flush=True)
    except Exception as e:  # not supported on this build
        print(json.dumps({"gemm": "torch._grouped_mm", "error": str(e)[:200]}), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
