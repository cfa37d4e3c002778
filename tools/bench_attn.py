"""Micro-benchmark: paged decode attention, Llama-3-8B shapes (32 q / 8 kv heads, d 128), 64
sequences, rotating over 4 layers' KV caches (> the 256 MiB Infinity Cache) like a real step."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from polykey_service_amd.ops import attention as A  # noqa: E402
from polykey_service_amd.ops import native  # noqa: E402

B, NQ, NKV, D, BS = 64, 32, 8, 128, 32
for ctx in (128, 384, 1024, 4096):
    maxb = (ctx + BS - 1) // BS
    nblk = B * maxb + 1
    layers = [(torch.randn(nblk, NKV, BS, D, device="cuda").to(torch.bfloat16),
               torch.randn(nblk, NKV, D, BS, device="cuda").to(torch.bfloat16)) for _ in range(4)]
    bt = torch.arange(B * maxb, dtype=torch.int32, device="cuda").view(B, maxb)
    cl = torch.full((B,), ctx, dtype=torch.int32, device="cuda")
    q = torch.randn(B, NQ, D, device="cuda").to(torch.bfloat16)
    o, ml = A.decode_workspace(B, NQ, maxb, BS, "cuda")
    md = A.AttnMetadata(num_decode=B, num_prefill=0, num_prefill_tokens=0, max_prefill_q_len=0,
                        slot_mapping=None, decode_block_tables=bt, decode_context_lens=cl,
                        decode_part_o=o, decode_part_ml=ml)
    row = f"ctx {ctx:5d}:"
    for z in (4, 16):
        native.lib().pk_set_decode_z(z)
        for i in range(4):
            A.paged_attention(q, *layers[i % 4], md, 0.088)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        n = 40
        e0.record()
        for i in range(n):
            A.paged_attention(q, *layers[i % 4], md, 0.088)
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) / n * 1000
        gb = B * ctx * NKV * D * 2 * 2 / 1e9
        row += f" | z{z} {us:7.1f} us {gb / us * 1e3:5.2f} TB/s"
    native.lib().pk_set_decode_z(4)
    print(row, flush=True)
    del layers
