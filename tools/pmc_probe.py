"""Tiny PMC sanity probe (one bf16 GEMM + the pk RMSNorm kernel): checks that rocprofv3 counter
collection works end to end on a box before a long profile."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from polykey_service_amd.ops import norm  # noqa: E402

x = torch.randn(256, 4096, device="cuda", dtype=torch.bfloat16)
w = torch.randn(4096, 4096, device="cuda", dtype=torch.bfloat16)
for _ in range(3):
    y = x @ w
    z = norm.rms_norm(y, torch.ones(4096, device="cuda", dtype=torch.bfloat16), 1e-5)
torch.cuda.synchronize()
print("pmc_probe ok", float(z.float().abs().mean()))
