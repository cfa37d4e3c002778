"""Probe: is the fused decode attention (8B shape, 64 sequences, ctx 384) faster when its K/V
cache lines were just read (Infinity Cache warm) than cold?  Decides whether prefetching a
layer's KV blocks during the HBM-light kernels before it (residual update, QKV GEMM) can pay.

Per iteration: stream a 512 MB unrelated buffer (flush), optionally read a fraction of the
layer's K / V cache (warm), then time only the attention launch with events (median of 40)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from polykey_service_amd.ops import attention as A
from polykey_service_amd.ops import gemm, reference

B, NQ, NKV, D, BS = 64, 32, 8, 128, 32
cs = reference.rope_cos_sin_cache(8192, 128, 500000.0, None, device="cuda")
flush = torch.empty(512 << 20, dtype=torch.uint8, device="cuda")
sink = torch.empty((), dtype=torch.bfloat16, device="cuda")
for ctx in (384, 512):
    per = (ctx + BS) // BS
    nblk = B * per + 8
    kc = torch.randn(nblk, NKV, BS, D, device="cuda").to(torch.bfloat16)
    vc = torch.randn(nblk, NKV, D, BS, device="cuda").to(torch.bfloat16)
    perm = torch.randperm(B * per, generator=torch.Generator().manual_seed(1)).to(torch.int32)
    bt = torch.zeros((B, 512), dtype=torch.int32)
    bt[:, :per] = perm.view(B, per)
    bt = bt.cuda()
    cl = torch.full((B,), ctx, dtype=torch.int32, device="cuda")
    pos = torch.full((B,), ctx - 1, dtype=torch.int32, device="cuda")
    slots = (bt[:, (ctx - 1) // BS] * BS + (ctx - 1) % BS).contiguous()
    md = A.AttnMetadata(num_decode=B, num_prefill=0, num_prefill_tokens=0, max_prefill_q_len=0,
                        slot_mapping=slots, decode_block_tables=bt, decode_context_lens=cl, decode_max_ctx=512)
    N = (NQ + 2 * NKV) * D
    p = gemm.Partial(torch.randn(4 * B * N, device="cuda") * 0.05, 4, B, N)
    res = {}
    for mode, frac in (("cold", 0.0), ("warm25", 0.25), ("warm50", 0.5), ("warm100", 1.0), ("cold2", 0.0)):
        ts = []
        for it in range(40):
            torch.amax(flush.view(torch.bfloat16), 0, out=sink)  # read-only flush (no dirty lines)
            if frac > 0:
                n = int(nblk * frac)
                torch.amax(kc[:n].view(-1), 0, out=sink)
                torch.amax(vc[:n].view(-1), 0, out=sink)
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            A.paged_decode_from_qkv(p, pos, cs, kc, vc, md, 0.088, NQ, NKV)
            e.record()
            torch.cuda.synchronize()
            ts.append(s.elapsed_time(e) * 1000)
        ts.sort()
        res[mode] = round(ts[len(ts) // 2], 2)
    print(f"ctx {ctx}: KV {2 * B * ctx * NKV * D * 2 / 1e6:.0f} MB  " + "  ".join(f"{k} {v} us" for k, v in res.items()),
          flush=True)
    del kc, vc
