"""LM-head decode GEMM (Llama-3 vocab 128256 x 4096, 64 rows, block-packed) with non-temporal weight
loads (production: streams >= gemm.NT_MIN_BYTES) against the default cache policy, event-timed over
two cold copies, alternating.   python tools/lm_head_nt_probe.py [rows]"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from polykey_service_amd.ops import gemm, native  # noqa: E402


def main():
    M = int(sys.argv[1]) if len(sys.argv) > 1 else 64
    N, K = 128256, 4096
    x = torch.randn(M, K, device="cuda").to(torch.bfloat16)
    wps = [gemm.pack_weight((torch.randn(N, K, device="cuda") * 0.02).to(torch.bfloat16)) for _ in range(2)]
    out = torch.empty(M, N, dtype=torch.bfloat16, device="cuda")

    def run(i, nt):
        mode = gemm.PACKED_BIT | (gemm.NT_BIT if nt else 0)
        native.call("pk_skinny_gemm", out.data_ptr(), 0, x.data_ptr(), wps[i % 2].data_ptr(), M, N, K, x.stride(0),
                    out.stride(0), 1, mode, native.stream_ptr())

    res = {}
    for _ in range(3):
        for nt in (True, False):
            for i in range(4):
                run(i, nt)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for i in range(20):
                run(i, nt)
            e1.record()
            torch.cuda.synchronize()
            res.setdefault("nt" if nt else "default", []).append(round(e0.elapsed_time(e1) / 20 * 1000, 1))
    print(json.dumps({"M": M, "us": res}), flush=True)


if __name__ == "__main__":
    main()
