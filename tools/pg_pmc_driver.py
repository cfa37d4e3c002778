"""One dense gate_up-shaped prefill GEMM per variant (argv, default 4) and hipBLASLt, a few calls each, for
a rocprofv3 --pmc pass (tools/gpu/pg_pmc.sh)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from polykey_service_amd.ops import gemm_prefill  # noqa: E402

M, N, K = 8192, 28672, 4096
x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
w = torch.randn(N, K, device="cuda", dtype=torch.bfloat16) * 0.02
out = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
for v in [int(a) for a in sys.argv[1:]] or (4,):
    for _ in range(3):
        gemm_prefill.linear(x, w, out=out, variant=v)
for _ in range(3):
    torch.mm(x, w.t(), out=out)
torch.cuda.synchronize()
