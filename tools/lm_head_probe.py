"""LM-head decode GEMM (Llama-3 vocab 128256 x 4096, bf16, block-packed, non-temporal loads) at
64 rows: the production tiling (1002 workgroups of 128-row n-blocks) against 64-row n-blocks
(2004 workgroups: a finer last wave on 256 CUs), event-timed over two cold copies, alternating.

    python tools/lm_head_probe.py [rows]
"""
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

    def run(i, half):
        wp = wps[i % 2]
        mode = 0 | gemm._wmode(wp) | (gemm.HALF_BIT if half else 0)
        native.call("pk_skinny_gemm", out.data_ptr(), 0, x.data_ptr(), wp.data_ptr(), M, N, K, x.stride(0),
                    out.stride(0), 1, mode, native.stream_ptr())

    res = {}
    for rep in range(3):
        for half in (False, True):
            for i in range(4):
                run(i, half)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for i in range(20):
                run(i, half)
            e1.record()
            torch.cuda.synchronize()
            res.setdefault("half" if half else "prod", []).append(round(e0.elapsed_time(e1) / 20 * 1000, 1))
    run(0, False)
    a = out.clone()
    run(0, True)
    torch.cuda.synchronize()
    print(json.dumps({"M": M, "us": res, "bit_identical": bool(torch.equal(a, out))}), flush=True)


if __name__ == "__main__":
    main()
