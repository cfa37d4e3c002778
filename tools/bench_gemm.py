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

# ---- fused decode-chain modes (8B shapes, M = 64, packed weights) vs the unfused kernel pairs
M, H, I, nq, nkv, bs = 64, 4096, 14336, 32, 8, 32
ctr = torch.zeros(4096, dtype=torch.int32, device="cuda")
res = torch.randn(M, H, device="cuda").to(torch.bfloat16)
parts = res.float().view(M, H // 128, 128).pow(2).sum(-1).t().contiguous()
nw = torch.ones(H, dtype=torch.bfloat16, device="cuda")
pos = torch.arange(M, dtype=torch.int32, device="cuda") + 300
cs = torch.randn(4096, 128, device="cuda")
slots = torch.arange(M, dtype=torch.int32, device="cuda") * 3
kc = torch.zeros(512, nkv, bs, 128, dtype=torch.bfloat16, device="cuda")
vc = torch.zeros(512, nkv, 128, bs, dtype=torch.bfloat16, device="cuda")
print("fused decode chain (us):", flush=True)
for name, N, K in (("qkv", (nq + 2 * nkv) * 128, H), ("o", H, H), ("gate_up", 2 * I, H), ("down", H, I)):
    n = max(2, (1 << 30) // (N * K * 2) + 1)
    wl = [gemm.pack_weight((torch.randn(N, K, device="cuda") * 0.02).to(torch.bfloat16)) for _ in range(n)]
    x = torch.randn(M, K, device="cuda").to(torch.bfloat16)
    S = gemm.choose_split(N, K, M)
    row = f"  {name:8s} S{S}"
    if name == "qkv":
        t0 = timeit(lambda i: gemm.qkv_reduce_rope_cache(gemm.linear_partial(x, wl[i], ws, S, packed=wl[i]), pos, cs,
                                                         kc, vc, slots, nq, nkv), n)
        t1 = timeit(lambda i: gemm.linear_qkv_rope(x, wl[i], ws, ctr, pos, cs, kc, vc, slots, nq, nkv, S,
                                                   packed=wl[i]), n)
        t2 = timeit(lambda i: gemm.linear_qkv_rope(res, wl[i], ws, ctr, pos, cs, kc, vc, slots, nq, nkv, S,
                                                   packed=wl[i], norm=gemm.NormIn(parts, nw, 1e-5)), n)
        row += f" partial+reduce_rope {t0:6.1f} | fused {t1:6.1f} | fused+norm {t2:6.1f}"
    elif name in ("o", "down"):
        r2 = res.clone()
        p2 = torch.empty(H // 128 * M, device="cuda")
        t0 = timeit(lambda i: gemm.partial_add_rms_norm(gemm.linear_partial(x, wl[i], ws, S, packed=wl[i]), r2, nw,
                                                        1e-5), n)
        t1 = timeit(lambda i: gemm.linear_add_residual(x, wl[i], ws, ctr, r2, p2, S, packed=wl[i]), n)
        row += f" partial+add_rmsnorm {t0:6.1f} | fused {t1:6.1f}"
    else:
        t0 = timeit(lambda i: gemm.linear_silu(x, wl[i], ws, packed=wl[i]), n)
        t1 = timeit(lambda i: gemm.linear_silu(res, wl[i], ws, packed=wl[i], norm=gemm.NormIn(parts, nw, 1e-5)), n)
        row += f" silu {t0:6.1f} | silu+norm {t1:6.1f}"
    print(row, flush=True)
    del wl
