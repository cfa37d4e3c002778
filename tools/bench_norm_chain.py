"""Micro-benchmark: the per-layer norm step of the decode chain (M = 64, H = 4096, split-K 8):
splitk_add_rmsnorm (residual += slabs; x = rmsnorm) vs residual_parts (residual += slabs; sums of
squares for the folded-norm consumer), and the gate_up GEMM with / without the row scale."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from polykey_service_amd.ops import gemm  # noqa: E402


def timeit(fn, iters=200):
    for _ in range(10):
        fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(20):
            fn()
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters // 20):
        g.replay()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters * 1000.0


M, H, S, I = 64, 4096, 8, 14336
res = torch.randn(M, H, device="cuda").to(torch.bfloat16)
ws = torch.randn(S * M * H, device="cuda") * 0.01
p = gemm.Partial(ws, S, M, H)
nw = torch.ones(H, device="cuda", dtype=torch.bfloat16)
buf = torch.zeros(4 * 64, device="cuda")
print(f"splitk_add_rmsnorm {timeit(lambda: gemm.partial_add_rms_norm(p, res, nw, 1e-5)):6.2f} us")
print(f"residual_parts     {timeit(lambda: gemm.residual_parts(p, res, buf)):6.2f} us")
wl = [gemm.pack_weight((torch.randn(2 * I, H, device='cuda') * 0.02).to(torch.bfloat16)) for _ in range(6)]
w0 = torch.empty(2 * I, H, device="cuda", dtype=torch.bfloat16)
parts = gemm.residual_parts(None, res, buf)
cnt = [0]


def gu(rowscale):
    cnt[0] += 1
    return gemm.linear_silu(res, w0, packed=wl[cnt[0] % 6], rowscale=gemm.RowScale(parts, 1e-5) if rowscale else None)


print(f"gate_up silu       {timeit(lambda: gu(False)):6.2f} us (6 weight copies rotated inside a graph)")
print(f"gate_up rowscale   {timeit(lambda: gu(True)):6.2f} us")
