"""Micro-benchmark: decode GEMM shapes, hand-written skinny kernel vs hipBLASLt (F.linear).

Weights rotate over enough copies (> 1 GiB) that nothing is served from the 256 MiB
Infinity Cache, matching a real decode step where every layer's weights are cold.
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import torch.nn.functional as F

from polykey_service_amd.ops import gemm

gemm.SKINNY_ENABLED = True


def timeit(fn, n, iters=40):
    for i in range(4):
        fn(i % n)
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for i in range(iters):
        fn(i % n)
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1000.0


shapes = [("qkv", 6144, 4096), ("o", 4096, 4096), ("gate_up", 28672, 4096), ("down", 4096, 14336),
          ("lm_head", 128256, 4096), ("70b_qkv", 1280, 8192), ("70b_o", 8192, 1024), ("70b_gu", 7168, 8192),
          ("70b_down", 8192, 3584)]
ws = torch.empty(16 * 64 * 131072, dtype=torch.float32, device="cuda")
for M in (int(a) for a in (sys.argv[1:] or ["64"])):
    print(f"M={M}", flush=True)
    for name, N, K in shapes:
        x = torch.randn(M, K, device="cuda").to(torch.bfloat16)
        bytes_ = N * K * 2
        n = max(2, (1 << 30) // bytes_ + 1)
        ws_list = [(torch.randn(N, K, device="cuda") * 0.02).to(torch.bfloat16) for _ in range(n)]
        tb = timeit(lambda i: F.linear(x, ws_list[i]), n)
        row = f"  {name:8s} N={N:6d} K={K:5d}  hipBLASLt {tb:7.1f}us {bytes_/tb/1e6:5.2f}TB/s"
        for S in (1, 2, 4, 8, 16):
            if K % (256 * S) or N % 128:
                continue
            if S == 1:
                ts = timeit(lambda i: gemm.linear(x, ws_list[i]), n)
            else:
                ts = timeit(lambda i: gemm.linear_partial(x, ws_list[i], ws, S), n)
            row += f" | S{S} {ts:6.1f}us {bytes_/ts/1e6:5.2f}"
        if name == "gate_up" or name == "70b_gu":
            ts = timeit(lambda i: gemm.linear_silu(x, ws_list[i], ws), n)
            row += f" | silu {ts:6.1f}us {bytes_/ts/1e6:5.2f}"
        wp_list = [gemm.pack_weight(w) for w in ws_list]
        for S in (1, 2, 4, 8, 16):
            if K % (256 * S) or N % 128:
                continue
            if S == 1:
                tn = timeit(lambda i: gemm.linear(x, ws_list[i], packed=wp_list[i]), n)
            else:
                tn = timeit(lambda i: gemm.linear_partial(x, ws_list[i], ws, S, packed=wp_list[i]), n)
            row += f" | PK-S{S} {tn:6.1f}us {bytes_/tn/1e6:5.2f}"
        if name in ("gate_up", "70b_gu"):
            tsd = timeit(lambda i: gemm.linear_silu(x, ws_list[i], ws, packed=wp_list[i]), n)
            row += f" | PK-silu {tsd:6.1f}us {bytes_/tsd/1e6:5.2f}"
        del wp_list
        print(row, flush=True)
        del ws_list
        torch.cuda.empty_cache()
