"""rope_and_cache at the 8B prefill step shape (8192 tokens = 32 sequences x 256, block 32)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from polykey_service_amd.ops import attention as A  # noqa: E402
from polykey_service_amd.ops import reference as ref  # noqa: E402

T, nq, nkv, bs = 8192, 32, 8, 32
qkv = torch.randn(T, (nq + 2 * nkv) * 128, device="cuda").to(torch.bfloat16)
pos = (torch.arange(T, dtype=torch.int32) % 256).cuda()
cs = ref.rope_cos_sin_cache(8192, 128, 500000.0, None, device="cuda")
nb = T // bs + 8
slots = torch.arange(T, dtype=torch.int32, device="cuda")
kc = torch.zeros(nb, nkv, bs, 128, dtype=torch.bfloat16, device="cuda")
vc = torch.zeros(nb, nkv, 128, bs, dtype=torch.bfloat16, device="cuda")
for _ in range(3):
    A.rope_and_cache(qkv, pos, cs, kc, vc, slots, nq, nkv)
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(50):
    A.rope_and_cache(qkv, pos, cs, kc, vc, slots, nq, nkv)
e1.record()
torch.cuda.synchronize()
print(f"rope_and_cache T={T}: {e0.elapsed_time(e1) * 1000 / 50:.1f} us/call")
