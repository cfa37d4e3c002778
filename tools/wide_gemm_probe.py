"""Wide-batch decode GEMMs (Llama-3-8B LM head 128256 x 4096, gate_up 28672 x 4096 + SiLU) at
128-512 rows: hipBLASLt (F.linear) vs the hand-written MFMA GEMM of prefill
(``ops/gemm_prefill.linear`` on the block-packed weight the decode path already holds) vs the
skinny decode GEMM.  Weights rotate over 4 copies so every call streams from HBM, as in a
decode step.  One JSON line per (op, rows, path): median us of 30 calls.

    python tools/wide_gemm_probe.py [rows ...]
"""
import json
import statistics
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, ".")
from polykey_service_amd.ops import gemm, gemm_prefill  # noqa: E402


def timed(fn, reps=30):
    for _ in range(3):
        fn(0)
    ts = []
    for i in range(reps):
        b, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        b.record()
        fn(i)
        e.record()
        e.synchronize()
        ts.append(b.elapsed_time(e) * 1e3)
    return statistics.median(ts)


def main(rows):
    dev = torch.device("cuda:0")
    torch.manual_seed(0)
    shapes = {"lm_head": (128256, 4096, 2), "gate_up": (28672, 4096, 4)}
    for op, (N, K, copies) in shapes.items():
        ws = [torch.randn(N, K, device=dev, dtype=torch.bfloat16) * 0.02 for _ in range(copies)]
        wp = [gemm.pack_weight(w) for w in ws]
        silu = op == "gate_up"
        for M in rows:
            x = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
            c = len(ws)
            if silu:
                blas = lambda i: gemm.silu_and_mul_interleaved(F.linear(x, ws[i % c]))  # noqa: E731
            else:
                blas = lambda i: F.linear(x, ws[i % c])  # noqa: E731
            mine = lambda i: gemm_prefill.linear(x, ws[i % c], silu=silu, packed=wp[i % c])  # noqa: E731
            ref = blas(0).float()
            got = mine(0).float()
            err = ((got - ref).abs().max() / ref.abs().max()).item()
            res = {"op": op, "M": M, "hipblaslt_us": round(timed(blas), 1), "mfma_packed_us": round(timed(mine), 1),
                   "rel_err": round(err, 5)}
            if not silu and M <= gemm.DECODE_MAX_M:
                res["skinny_us"] = round(timed(lambda i: gemm.linear(x, ws[i % c], packed=wp[i % c],
                                                                     max_m=gemm.DECODE_MAX_M)), 1)
            print(json.dumps(res), flush=True)
        del ws, wp
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main([int(a) for a in sys.argv[1:]] or [128, 192, 256, 384, 512])
