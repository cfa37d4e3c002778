"""A/B of two prefill GEMM variants in one process, alternating, median of rounds (guide §5.4:
compare schedules in one process on random data).  python tools/prefill_gemm_ab.py [va] [vb] (default: the 8-wave kernel 4 against the 4-wave kernel 6, plus the hipBLASLt column)"""
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from polykey_service_amd.ops import gemm_prefill  # noqa: E402


def t(fn, reps=10):
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
    va, vb = (int(sys.argv[1]), int(sys.argv[2])) if len(sys.argv) > 2 else (4, 6)
    torch.manual_seed(0)
    dev = "cuda"
    cases = []
    for name, M, N, K in [("qkv", 8192, 6144, 4096), ("gate_up", 8192, 28672, 4096), ("down", 8192, 4096, 14336),
                          ("o16k", 16384, 4096, 4096)]:
        x = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
        w = torch.randn(N, K, device=dev, dtype=torch.bfloat16) * 0.02
        out = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        cases.append((name, 2.0 * M * N * K, lambda v, x=x, w=w, out=out: gemm_prefill.linear(x, w, out=out, variant=v),
                      lambda x=x, w=w, out=out: torch.mm(x, w.t(), out=out)))
    E, H, I = 8, 4096, 14336
    counts = [2048 + d for d in (40, -30, 12, -25, 0, 31, -16, -12)]
    T = sum(counts)
    offs = torch.tensor([0] + list(torch.tensor(counts).cumsum(0)), dtype=torch.int32, device=dev)
    x = torch.randn(T, H, device=dev, dtype=torch.bfloat16)
    w13 = torch.randn(E, 2 * I, H, device=dev, dtype=torch.bfloat16) * 0.02
    h = torch.randn(T, I, device=dev, dtype=torch.bfloat16)
    w2 = torch.randn(E, H, I, device=dev, dtype=torch.bfloat16) * 0.02
    # hipBLASLt reference for the grouped cases: torch._grouped_mm over the same device offsets
    # (no SiLU epilogue: it would need a separate pass)
    gm = getattr(torch, "_grouped_mm", None)
    offs_end = offs[1:].contiguous()
    blas13 = (lambda: gm(x, w13.transpose(1, 2), offs=offs_end)) if gm else None
    blas2 = (lambda: gm(h, w2.transpose(1, 2), offs=offs_end)) if gm else None
    cases.append(("moe_w13_silu", 2.0 * T * 2 * I * H,
                  lambda v: gemm_prefill.grouped_linear(x, w13, offs, silu=True, variant=v), blas13))
    cases.append(("moe_w2", 2.0 * T * H * I, lambda v: gemm_prefill.grouped_linear(h, w2, offs, variant=v), blas2))
    for name, fl, fn, blas in cases:
        ra, rb, rc = [], [], []
        for _ in range(5):
            ra.append(t(lambda: fn(va)))
            rb.append(t(lambda: fn(vb)))
            if blas is not None:
                try:
                    rc.append(t(blas))
                except Exception:  # noqa: BLE001 - reference column only
                    blas = None
        ma, mb = statistics.median(ra), statistics.median(rb)
        row = {"gemm": name, f"v{va}_us": round(ma, 1), f"v{vb}_us": round(mb, 1),
               f"v{va}_tfs": round(fl / ma / 1e6), f"v{vb}_tfs": round(fl / mb / 1e6),
               "gain_pct": round(100 * (ma / mb - 1), 1)}
        if rc:
            mc = statistics.median(rc)
            row.update({"hipblaslt_us": round(mc, 1), "hipblaslt_tfs": round(fl / mc / 1e6),
                        f"v{vb}_vs_hipblaslt_pct": round(100 * (mb / mc - 1), 1)})
        print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
