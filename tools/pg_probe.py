"""Time prefill GEMM variants at the Llama-3-8B gate_up shape (8192 x 28672 x 4096) and the
Mixtral grouped w2 in THIS process's kernel library (POLYKEY_LIB_LIBPK_KERNELS selects a
tools/lab/build_variant.py build): one JSON line per variant.  Used for ablations of the 4-wave
kernel (lab variants that drop one part of the k-loop: the timing shows what that part costs).
    python tools/pg_probe.py 6 4"""
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from polykey_service_amd.ops import gemm_prefill  # noqa: E402


def t(fn, reps=10):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    b.synchronize()
    return a.elapsed_time(b) * 1e3 / reps


def main():
    torch.manual_seed(0)
    lib = os.path.basename(os.environ.get("POLYKEY_LIB_LIBPK_KERNELS", "production"))
    M, N, K = 8192, 28672, 4096
    x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
    w = torch.randn(N, K, device="cuda", dtype=torch.bfloat16) * 0.02
    out = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    from polykey_service_amd.ops import gemm
    wp = gemm.pack_weight(w)  # odd variants read the block-packed copy
    for v in [int(a) for a in sys.argv[1:]] or [4]:
        kw = {"packed": wp} if v % 2 else {}
        us = statistics.median(t(lambda: gemm_prefill.linear(x, w, out=out, variant=v, **kw)) for _ in range(5))
        print(json.dumps({"lib": lib, "variant": v, "gate_up_us": round(us, 1),
                          "tfs": round(2.0 * M * N * K / us / 1e6)}), flush=True)


if __name__ == "__main__":
    main()
