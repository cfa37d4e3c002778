"""Micro-benchmark: paged causal prefill attention, Llama-3-8B heads (32 q / 8 kv, d 128, block 32):
the LDS-tiled kernel (K/V tiles shared by the GQA group's waves) vs the per-wave streaming kernel.
Reports us per call and causal TFLOP/s (4 * d * sum_i keys_i * heads)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from polykey_service_amd.ops import attention as A  # noqa: E402
from polykey_service_amd.ops import native  # noqa: E402

NQ, NKV, D, BS = 32, 8, 128, 32
for n_seqs, qlen, prefix in ((32, 256, 0), (8, 1024, 0), (2, 4096, 0), (16, 256, 1024)):
    ctx = prefix + qlen
    maxb = (ctx + BS - 1) // BS
    nblk = n_seqs * maxb + 1
    kc = torch.randn(nblk, NKV, BS, D, device="cuda").to(torch.bfloat16)
    vc = torch.randn(nblk, NKV, D, BS, device="cuda").to(torch.bfloat16)
    bt = torch.randperm(n_seqs * maxb, device="cuda").to(torch.int32).view(n_seqs, maxb)
    cl = torch.full((n_seqs,), ctx, dtype=torch.int32, device="cuda")
    cu = torch.arange(n_seqs + 1, dtype=torch.int32, device="cuda") * qlen
    q = torch.randn(n_seqs * qlen, NQ, D, device="cuda").to(torch.bfloat16)
    md = A.AttnMetadata(num_decode=0, num_prefill=n_seqs, num_prefill_tokens=n_seqs * qlen, max_prefill_q_len=qlen,
                        slot_mapping=None, prefill_block_tables=bt, prefill_context_lens=cl, prefill_cu_q=cu)
    keys = sum(prefix + i + 1 for i in range(qlen)) * n_seqs
    flops = 4.0 * D * keys * NQ
    row = f"{n_seqs:3d} seqs x {qlen:5d} q (+{prefix} cached):"
    for _ in range(3):
        A.paged_attention(q, kc, vc, md, 0.088)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(10):
        A.paged_attention(q, kc, vc, md, 0.088)
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) / 10 * 1000
    print(row + f" {us:8.1f} us {flops / us / 1e6:6.0f} TF/s", flush=True)

