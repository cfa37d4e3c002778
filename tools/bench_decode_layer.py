"""Micro-benchmark of the attention half of a decode layer (Llama-3-8B shapes, 64 sequences):
QKV split-K slabs → (a) reduce+RoPE+cache kernel then attention, or (b) attention fed by the
slabs directly (paged_decode_from_qkv).  Four layers' KV caches rotate (cold like a real step)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from polykey_service_amd.ops import attention as A  # noqa: E402
from polykey_service_amd.ops import gemm  # noqa: E402
from polykey_service_amd.ops import reference as ref  # noqa: E402

B, NQ, NKV, D, BS, S = 64, 32, 8, 128, 32, 4
N = (NQ + 2 * NKV) * D
for ctx in (128, 384, 1024):
    maxb = (ctx + BS) // BS + 1
    nblk = B * maxb + 1
    layers = [(torch.randn(nblk, NKV, BS, D, device="cuda").to(torch.bfloat16),
               torch.randn(nblk, NKV, D, BS, device="cuda").to(torch.bfloat16)) for _ in range(4)]
    bt = torch.arange(B * maxb, dtype=torch.int32, device="cuda").view(B, maxb)
    cl = torch.full((B,), ctx, dtype=torch.int32, device="cuda")
    pos = cl - 1
    slots = bt[:, (ctx - 1) // BS] * BS + (ctx - 1) % BS
    ws = torch.randn(S * B * N, device="cuda") * 0.1
    p = gemm.Partial(ws, S, B, N)
    cs = ref.rope_cos_sin_cache(8192, D, 500000.0).cuda()
    po, pml = A.decode_workspace(B, NQ, maxb, BS, "cuda")
    md = A.AttnMetadata(num_decode=B, num_prefill=0, num_prefill_tokens=0, max_prefill_q_len=0, slot_mapping=slots,
                        decode_block_tables=bt, decode_context_lens=cl, decode_part_o=po, decode_part_ml=pml,
                        decode_max_ctx=512 if ctx + 1 <= 512 else 0)  # short-context graphs

    def unfused(i):
        kc, vc = layers[i % 4]
        q = gemm.qkv_reduce_rope_cache(p, pos, cs, kc, vc, slots, NQ, NKV)
        return A.paged_attention(q, kc, vc, md, 0.088)

    def fused(i):
        kc, vc = layers[i % 4]
        return A.paged_decode_from_qkv(p, pos, cs, kc, vc, md, 0.088, NQ, NKV)

    row = f"ctx {ctx:5d}:"
    for name, fn in (("reduce+attn", unfused), ("fused", fused)):
        for i in range(4):
            fn(i)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for i in range(40):
            fn(i)
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) / 40 * 1000
        row += f" | {name} {us:7.1f} us {B * ctx * NKV * D * 4 / us / 1e6:5.2f} TB/s"
    print(row, flush=True)
    del layers
