"""Mixtral decode expert GEMMs in isolation (64 tokens x top-2 over 8 experts, block-packed
experts, 4 rotating weight sets so every call streams cold): w13 (+SiLU) and w2 at split-K
S = 1 / 2 / 4 (w2 as fp32 slabs for S > 1).  us per call and TB/s of expert weights."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from polykey_service_amd.ops import gemm, moe  # noqa: E402


def timeit(fn, iters=40):
    for i in range(4):
        fn(i)
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for i in range(iters):
        fn(i)
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) * 1e3 / iters


E, H, I, T, k = 8, 4096, 14336, 64, 2
g = torch.Generator(device="cuda").manual_seed(0)
sets = []
for _ in range(3):
    w13 = (torch.randn(E, 2 * I, H, device="cuda", generator=g) * 0.02).to(torch.bfloat16)
    w2 = (torch.randn(E, H, I, device="cuda", generator=g) * 0.02).to(torch.bfloat16)
    sets.append((w13, gemm.pack_weight(w13.view(-1, H)).view(w13.shape), w2, gemm.pack_weight(w2.view(-1, I)).view(w2.shape)))
    del w13, w2
x = torch.randn(T, H, device="cuda", generator=g).to(torch.bfloat16)
router = torch.randn(E, H, device="cuda", generator=g).to(torch.bfloat16) * 0.1
ids, wts = moe.topk_softmax(torch.nn.functional.linear(x, router), k)
off, srt, inv = moe.align(ids, E, 0, E)
h = torch.randn(T * k, I, device="cuda", generator=g).to(torch.bfloat16)
ws = torch.empty(4 * T * k * H, dtype=torch.float32, device="cuda")
res = {}
res["w13_silu_us"] = round(timeit(lambda i: gemm.grouped_linear(
    x, sets[i % 3][0], off, T, True, packed=sets[i % 3][1], a_rows=srt, a_row_div=k, n_rows=T * k)), 1)
for S in (1, 2, 4):
    res[f"w2_S{S}_us"] = round(timeit(lambda i, S=S: gemm.grouped_linear(
        h, sets[i % 3][2], off, T, False, packed=sets[i % 3][3], ws=ws, S=S)), 1)
gb13, gb2 = E * 2 * I * H * 2 / 1e9, E * H * I * 2 / 1e9
res["w13_TBs"] = round(gb13 / res["w13_silu_us"] * 1e3, 2)
res["w2_S1_TBs"] = round(gb2 / res["w2_S1_us"] * 1e3, 2)
print(json.dumps(res), flush=True)
