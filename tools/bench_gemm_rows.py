"""Decode GEMMs above 64 rows: the row-tiled weight-streaming kernel vs hipBLASLt (torch.mm).

8B projection shapes, M = 64 / 128 / 256 / 512, packed weights rotated over > 1 GiB of copies
(cold, as in a decode step).  For the row-tiled kernel the split is the default
(``gemm.choose_split``: row tiles replace K splits) and 2x / 0.5x of it.  One JSON line per
(shape, M) -> the decode chain's limits (``gemm.DECODE_MAX_M``, LM head / gate_up switches;
profiles/r3_decode_rows.txt).
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from polykey_service_amd.ops import gemm, native


def timeit(fn, n, iters=30):
    for i in range(3):
        fn(i % n)
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for i in range(iters):
        fn(i % n)
    e.record()
    torch.cuda.synchronize()
    return round(s.elapsed_time(e) / iters * 1000.0, 2)


SHAPES = [("qkv", 6144, 4096), ("o", 4096, 4096), ("gate_up", 28672, 4096), ("down", 4096, 14336),
          ("lm_head", 128256, 4096)]
Ms = [int(a) for a in sys.argv[1:]] or [64, 128, 256, 512]
ws = torch.empty(8 * 512 * 28672, dtype=torch.float32, device="cuda")
for name, N, K in SHAPES:
    nbytes = N * K * 2
    n = max(2, (1 << 30) // nbytes + 1)
    wl = [(torch.randn(N, K, device="cuda") * 0.02).to(torch.bfloat16) for _ in range(n)]
    pl = [gemm.pack_weight(w) for w in wl]
    for M in Ms:
        x = torch.randn(M, K, device="cuda").to(torch.bfloat16)
        out = torch.empty(M, N, dtype=torch.bfloat16, device="cuda")
        row = {"shape": name, "N": N, "K": K, "M": M}
        row["hipblaslt_us"] = timeit(lambda i: torch.mm(x, wl[i].t(), out=out), n)
        if name == "gate_up":  # S = 1 with the SiLU epilogue (hipBLASLt: the GEMM alone)
            row["skinny_us"] = timeit(lambda i: gemm.linear_silu(x, wl[i], ws, packed=pl[i],
                                                                 max_m=gemm.DECODE_MAX_M), n)
        elif name == "lm_head":
            row["skinny_us"] = timeit(lambda i: gemm.linear(x, wl[i], out=out, packed=pl[i],
                                                            max_m=gemm.DECODE_MAX_M), n)
        else:
            S0 = gemm.choose_split(N, K, M)
            for S in sorted({max(1, S0 // 2), S0, min(16, 2 * S0)}):
                if K % (256 * S) == 0 and S * M * N <= ws.numel():
                    row[f"skinny_S{S}_us"] = timeit(lambda i: gemm.linear_partial(x, wl[i], ws, S, packed=pl[i]), n)
        if M > 64:  # the same launch in 64-row tiles (W shared through the XCD L2) instead of 128
            S0 = 1 if name in ("gate_up", "lm_head") else gemm.choose_split(N, K, M)
            mode = {"gate_up": gemm.MODE_SILU, "lm_head": gemm.MODE_BF16}.get(name, gemm.MODE_PARTIAL)
            o = out if name != "gate_up" else torch.empty(M, N // 2, dtype=torch.bfloat16, device="cuda")
            row[f"skinny_rows64_S{S0}_us"] = timeit(lambda i: native.call(
                "pk_skinny_gemm", o.data_ptr(), ws.data_ptr(), x.data_ptr(), pl[i].data_ptr(), M, N, K, K,
                o.stride(0), S0, mode | gemm.PACKED_BIT | gemm.ROWS64_BIT, native.stream_ptr()), n)
        row["weight_tbs_best"] = round(nbytes / min(v for k, v in row.items() if k.endswith("_us")) / 1e6, 2)
        print(json.dumps(row), flush=True)
    del wl, pl
    torch.cuda.empty_cache()
