"""Decode GEMM n-block height probe at the gate_up shape (M 64, N 28672, K 4096, block-packed W,
4 rotating weight copies so every call streams cold): 128-row n-blocks (KR 2, 224 workgroups,
the SiLU epilogue's layout) vs 64-row n-blocks (KR 1, 448 workgroups), with / without
non-temporal loads.  Prints us per call."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from polykey_service_amd.ops import gemm, native  # noqa: E402


def timeit(fn, iters=60):
    for _ in range(5):
        fn(0)
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for i in range(iters):
        fn(i)
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) * 1e3 / iters


def main():
    M, K = 64, 4096
    for N in (28672, 14336 * 2 // 2, 6144, 4096):
        ws = [gemm.pack_weight((torch.randn(N, K, device="cuda") * 0.02).to(torch.bfloat16)) for _ in range(4)]
        x = torch.randn(M, K, device="cuda").to(torch.bfloat16)
        out = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
        slab = torch.empty(M * N, device="cuda", dtype=torch.float32)
        res = {}
        for name, mode, S in (("bf16_kr2_nt", 0 | 16 | 64, 1), ("bf16_kr2", 0 | 16, 1), ("part_kr2", 1 | 16, 1),
                              ("part_kr1", 1 | 16 | 128, 1), ("silu_kr2_nt", 2 | 16 | 64, 1)):
            o = out if mode & 7 != 1 else None

            def f(i, mode=mode, S=S, o=o):
                native.call("pk_skinny_gemm", o.data_ptr() if o is not None else 0, slab.data_ptr(), x.data_ptr(),
                            ws[i % 4].data_ptr(), M, N, K, K, N, S, mode, native.stream_ptr())
            res[name] = round(timeit(f), 2)
        gb = N * K * 2 / 1e9
        print({"N": N, "K": K, "GB": round(gb, 3), **res,
               "best_TBs": round(gb / min(res.values()) * 1e6 / 1e3, 2)}, flush=True)


if __name__ == "__main__":
    main()
