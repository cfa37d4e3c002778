"""Does the activation row stride matter to the 4-wave prefill GEMM (L1 / L2 channel conflicts of
8 KiB-strided rows)?  gate_up 8192 x 28672 x 4096 with x contiguous (lda 4096) vs padded rows
(lda 4096 + pad), against hipBLASLt on the same operands.  python tools/prefill_stride_probe.py"""
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
    M, N, K = 8192, 28672, 4096
    w = torch.randn(N, K, device="cuda", dtype=torch.bfloat16) * 0.02
    out = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    ref = None
    for pad in (0, 64, 128, 256):
        base = torch.randn(M, K + pad, device="cuda", dtype=torch.bfloat16)
        x = base[:, :K]
        if ref is None:
            x0 = x.contiguous()
        else:
            x.copy_(x0)
        ours = min(t(lambda: gemm_prefill.linear(x, w, out=out)) for _ in range(3))
        y = out.clone()
        blas = min(t(lambda: torch.mm(x, w.t(), out=out)) for _ in range(3))
        if ref is None:
            ref = y
        print(json.dumps({"lda": K + pad, "v6_us": round(ours, 1), "hipblaslt_us": round(blas, 1),
                          "same_bits": bool(torch.equal(y, ref))}), flush=True)


if __name__ == "__main__":
    main()
