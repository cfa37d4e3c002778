"""One prefill-attention case for PMC runs: 2 sequences x 4096 causal queries, Llama-3-8B heads
(32 q / 8 kv, d 128, block 32), implementation from argv[1] (pk_set_prefill_impl), 5 calls."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from polykey_service_amd.ops import attention as A  # noqa: E402
from polykey_service_amd.ops import native  # noqa: E402

impl = int(sys.argv[1]) if len(sys.argv) > 1 else 2
NQ, NKV, D, BS, n_seqs, qlen = 32, 8, 128, 32, 2, 4096
maxb = (qlen + BS - 1) // BS
kc = torch.randn(n_seqs * maxb + 1, NKV, BS, D, device="cuda").to(torch.bfloat16)
vc = torch.randn(n_seqs * maxb + 1, NKV, D, BS, device="cuda").to(torch.bfloat16)
bt = torch.randperm(n_seqs * maxb, device="cuda").to(torch.int32).view(n_seqs, maxb)
cl = torch.full((n_seqs,), qlen, dtype=torch.int32, device="cuda")
cu = torch.arange(n_seqs + 1, dtype=torch.int32, device="cuda") * qlen
q = torch.randn(n_seqs * qlen, NQ, D, device="cuda").to(torch.bfloat16)
md = A.AttnMetadata(num_decode=0, num_prefill=n_seqs, num_prefill_tokens=n_seqs * qlen, max_prefill_q_len=qlen,
                    slot_mapping=None, prefill_block_tables=bt, prefill_context_lens=cl, prefill_cu_q=cu)
native.lib().pk_set_prefill_impl(impl)
for _ in range(5):
    A.paged_attention(q, kc, vc, md, 0.088)
torch.cuda.synchronize()
print("ok", impl)
