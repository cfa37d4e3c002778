"""Decode GEMMs at 256 / 512 rows (Llama-3-8B shapes, cold weights rotated over 4 copies):
hipBLASLt (torch.mm) vs the skinny decode GEMM's XCD-grouped 128-row tiles, each at the split the
decode chain uses (gate_up: the folded-norm SiLU launch, S = 1).  One JSON line per shape and row
count.  (The 256-row MT = 16 tiles it also timed in round 4 were slower and are gone:
profiles/r4_wide_tiles_probe.jsonl.)"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from polykey_service_amd.ops import gemm  # noqa: E402

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
        ws_ = [(torch.randn(N, K, device=d) * 0.02).to(torch.bfloat16) for _ in range(L)]
        wp = [gemm.pack_weight(w) for w in ws_]
        for M in (256, 512):
            x = torch.randn(M, K, device=d).to(torch.bfloat16)
            out = torch.empty(M, N, dtype=torch.bfloat16, device=d)
            slab = torch.empty(16 * M * N, dtype=torch.float32, device=d)
            parts = gemm.residual_parts(None, x.clone(), torch.empty((K // gemm.PART_COLS) * M, device=d))
            rs = gemm.RowScale(parts.view(-1, M), 1e-5)
            row = {"shape": name, "M": M, "N": N, "K": K}
            row["hipblaslt_us"] = timeit(lambda i: torch.mm(x, ws_[i % L].t(), out=out))
            if name == "gate_up":
                fn = lambda i: gemm.linear_silu(x, ws_[i % L], packed=wp[i % L], rowscale=rs)  # noqa: E731
            else:
                fn = lambda i: gemm.linear_partial(x, ws_[i % L], slab, packed=wp[i % L])  # noqa: E731
            try:
                row["rows128_us"] = timeit(fn)
            except Exception as e:  # noqa: BLE001 - a probe: report and go on
                row["rows128_us"] = f"error: {e}"
            flops = 2.0 * M * N * K
            for k in ("hipblaslt_us", "rows128_us"):
                if isinstance(row[k], float):
                    row[k.replace("_us", "_tfs")] = round(flops / row[k] / 1e6, 1)
            print(json.dumps(row), flush=True)
        del ws_, wp


if __name__ == "__main__":
    main()
