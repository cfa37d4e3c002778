"""Decode GEMMs at 256 / 512 rows (Llama-3-8B shapes, cold weights rotated over 4 copies):
hipBLASLt (F.linear) vs the hand-written MFMA prefill GEMM (256 x 256 tiles, block-packed W,
csrc/kernels/gemm_prefill.hip) vs the row-tiled skinny decode GEMM.  One JSON line per shape."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from polykey_service_amd.ops import gemm  # noqa: E402
from polykey_service_amd.ops import gemm_prefill  # noqa: E402

SHAPES = {"qkv": (6144, 4096), "o": (4096, 4096), "gate_up": (28672, 4096), "down": (4096, 14336)}
L = 4


def timeit(fn, n=30):
    for i in range(L):
        fn(i)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for i in range(n):
        fn(i)
    e1.record()
    torch.cuda.synchronize()
    return round(e0.elapsed_time(e1) * 1000 / n, 2)


def main():
    d = "cuda"
    for name, (N, K) in SHAPES.items():
        ws = [(torch.randn(N, K, device=d) * 0.02).to(torch.bfloat16) for _ in range(L)]
        wp = [gemm.pack_weight(w) for w in ws]
        for M in (256, 512):
            x = torch.randn(M, K, device=d).to(torch.bfloat16)
            out = torch.empty(M, N, dtype=torch.bfloat16, device=d)
            flops = 2.0 * M * N * K
            row = {"shape": name, "M": M, "N": N, "K": K}
            row["hipblaslt_us"] = timeit(lambda i: torch.mm(x, ws[i % L].t(), out=out))
            try:
                row["prefill_mfma_us"] = timeit(lambda i: gemm_prefill.linear(x, ws[i % L], out=out,
                                                                               packed=wp[i % L]))
            except Exception as e:  # noqa: BLE001 - a probe: report and go on
                row["prefill_mfma_us"] = f"error: {e}"
            try:
                row["skinny_us"] = timeit(lambda i: gemm.linear(x, ws[i % L], packed=wp[i % L],
                                                                max_m=gemm.DECODE_MAX_M))
            except Exception as e:  # noqa: BLE001
                row["skinny_us"] = f"error: {e}"
            for k in ("hipblaslt_us", "prefill_mfma_us", "skinny_us"):
                if isinstance(row[k], float):
                    row[k.replace("_us", "_tfs")] = round(flops / row[k] / 1e6, 1)
            print(json.dumps(row), flush=True)
        del ws, wp


if __name__ == "__main__":
    main()
