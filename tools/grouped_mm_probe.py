"""torch._grouped_mm on ROCm at the Mixtral prefill expert shapes with ragged (non-aligned)
expert row counts: correctness vs a per-expert loop, and time vs the hand-written grouped GEMM."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from polykey_service_amd.ops import gemm, gemm_prefill  # noqa: E402


def t(fn, reps=5):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    b.synchronize()
    return a.elapsed_time(b) * 1e3 / reps


torch.manual_seed(0)
E, H, I = 8, 4096, 14336
counts = [2048 + d for d in (37, -29, 11, -23, 3, 29, -17, -11)]
T = sum(counts)
offs = torch.tensor([0] + list(torch.tensor(counts).cumsum(0)), dtype=torch.int32, device="cuda")
x = torch.randn(T, H, device="cuda", dtype=torch.bfloat16)
w13 = torch.randn(E, 2 * I, H, device="cuda", dtype=torch.bfloat16) * 0.02
w2 = torch.randn(E, H, I, device="cuda", dtype=torch.bfloat16) * 0.02
h = torch.randn(T, I, device="cuda", dtype=torch.bfloat16)
o32 = offs[1:].contiguous()
res = {}
try:
    y = torch._grouped_mm(x, w13.transpose(1, 2), offs=o32)
    lo = 0
    err = 0.0
    for e, c in enumerate(counts):
        ref = x[lo:lo + c].float() @ w13[e].float().t()
        err = max(err, (y[lo:lo + c].float() - ref).abs().max().item())
        lo += c
    res["grouped_mm_w13_maxerr"] = round(err, 4)
    res["grouped_mm_w13_us"] = round(t(lambda: torch._grouped_mm(x, w13.transpose(1, 2), offs=o32)), 1)
    yy = torch.empty(T, I, device="cuda", dtype=torch.bfloat16)
    res["grouped_mm_w13_silu_us"] = round(t(lambda: gemm.silu_and_mul_interleaved(
        torch._grouped_mm(x, w13.transpose(1, 2), offs=o32), out=yy)), 1)
    res["grouped_mm_w2_us"] = round(t(lambda: torch._grouped_mm(h, w2.transpose(1, 2), offs=o32)), 1)
except Exception as ex:  # noqa: BLE001
    res["grouped_mm_error"] = str(ex)[:300]
res["pk4_w13_silu_us"] = round(t(lambda: gemm_prefill.grouped_linear(x, w13, offs, silu=True, variant=4)), 1)
res["pk4_w2_us"] = round(t(lambda: gemm_prefill.grouped_linear(h, w2, offs, variant=4)), 1)
print(json.dumps(res), flush=True)
