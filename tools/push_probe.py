"""GEMM-side cost of the push epilogue (gemm.push_projection, MODE_PUSH) at the 70B TP=8 per-rank
o / down shapes, one process on one GPU: the "peers" are 8 local stand-in IPC buffers (signals +
slots, laid out as custom_allreduce.hip's), so the pushes are local stores -- the xGMI time they
would hide is not measured here.  Per shape: a graph of 80 back-to-back launches of the plain
split-K GEMM (the slabs the fused collective reduces) vs the push GEMM (last split of each n-block
sums the slabs, stores the bf16 tile into its owner's slot, stamps the owner's flag).

    python tools/push_probe.py
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from polykey_service_amd.ops import gemm, native  # noqa: E402
from polykey_service_amd.parallel import custom_ar  # noqa: E402


def timed(fn, reps=5):
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        fn()
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    with torch.cuda.graph(g):
        for _ in range(80):
            fn()
    best = 1e9
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        g.replay()
        e1.record()
        torch.cuda.synchronize()
        best = min(best, e0.elapsed_time(e1))
    return round(best * 1000 / 80, 2)


def main():
    dev = torch.device("cuda:0")
    W, M, N = 8, 64, 8192
    sig = custom_ar._lib().pk_car_sig_bytes()
    slot = M * N * 2
    bufs = [torch.zeros(sig + 4 * slot, dtype=torch.uint8, device=dev) for _ in range(W)]
    peers = torch.tensor([b.data_ptr() for b in bufs], dtype=torch.int64, device=dev)
    tgt = gemm.PushTarget(peers.data_ptr(), 0, W, slot)
    ctr = torch.zeros(N // 64, dtype=torch.int32, device=dev)
    out = []
    for name, K, down in (("o", 1024, False), ("down", 3584, True)):
        x = torch.randn(M, K, device=dev).to(torch.bfloat16)
        w = (torch.randn(N, K, device=dev) * 0.05).to(torch.bfloat16)
        wp = gemm.pack_weight(w)
        ws = torch.empty(8 * M * N, dtype=torch.float32, device=dev)
        plain = (lambda: gemm.linear_down(x, w, ws, wp)) if down else \
            (lambda: gemm.linear_partial(x, w, ws, packed=wp, half=True))
        push = lambda: gemm.push_projection(x, w, ws, wp, ctr, tgt, down=down)  # noqa: E731
        push1 = lambda: gemm.push_projection(x, w, ws, wp, ctr, tgt, down=down, split=1)  # noqa: E731
        plain1 = lambda: native.call("pk_skinny_gemm", 0, ws.data_ptr(), x.data_ptr(), wp.data_ptr(), M, N, K,  # noqa: E731
                                     K, N, 1, 1 | gemm.PACKED_BIT | gemm.HALF_BIT, native.stream_ptr())
        r = {"proj": name, "M": M, "N": N, "K": K, "lib": os.environ.get("POLYKEY_LIB_LIBPK_KERNELS", "in-tree"),
             "plain_us": timed(plain), "push_us": timed(push), "plain_s1_us": timed(plain1), "push_s1_us": timed(push1)}
        r["push_minus_plain_us"] = round(r["push_us"] - r["plain_us"], 2)
        assert int(ctr.abs().sum()) == 0
        out.append(r)
        print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
