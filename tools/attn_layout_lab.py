"""A/B of decode-attention builds loaded side by side (labbin/libattn_*.so, each a standalone
build of csrc/kernels/attention.hip with different -D switches), interleaved rounds in one
process at the 8B bench shape (64 seqs, 32 q / 8 kv heads, block 32):

    python tools/attn_layout_lab.py --libs base,kfrag [--ctx 256,384,512]
"""
import argparse
import ctypes
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from polykey_service_amd.ops import reference  # noqa: E402

P, I32, F32 = ctypes.c_void_p, ctypes.c_int, ctypes.c_float
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def load(tag):
    lib = ctypes.CDLL(os.path.join(ROOT, "labbin", f"libattn_{tag}.so"))
    f = lib.pk_paged_decode
    f.argtypes = [P, P, P, P, P, P, P, P, P, I32, I32, I32, I32, I32, I32, I32, F32, I32, P]
    g = lib.pk_paged_decode_qkv
    g.argtypes = [P, P, I32, I32, P, P, P, P, P, P, P, P, P, I32, I32, I32, I32, I32, I32, F32, I32, P]
    return f, g


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--libs", default="base,kfrag")
    ap.add_argument("--ctx", default="256,384,512")
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--rounds", type=int, default=5)
    a = ap.parse_args()
    libs = {t: load(t) for t in a.libs.split(",")}
    B, NQ, NKV, D, BS = 64, 32, 8, 128, 32
    cs = reference.rope_cos_sin_cache(8192, 128, 500000.0, None, device="cuda")
    st = lambda: ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    for ctx in (int(c) for c in a.ctx.split(",")):
        maxb = 16384 // BS
        per = (ctx + BS) // BS
        nblk = B * per + 8
        g = torch.Generator(device="cuda").manual_seed(0)
        layers = [(torch.randn(nblk, NKV, BS, D, device="cuda", generator=g).to(torch.bfloat16),
                   torch.randn(nblk, NKV, D, BS, device="cuda", generator=g).to(torch.bfloat16)) for _ in range(4)]
        perm = torch.randperm(B * per, generator=torch.Generator().manual_seed(1)).to(torch.int32)
        bt = torch.zeros((B, maxb), dtype=torch.int32)
        bt[:, :per] = perm.view(B, per)
        bt = bt.cuda()
        cl = torch.full((B,), ctx, dtype=torch.int32, device="cuda")
        pos = torch.full((B,), ctx - 1, dtype=torch.int32, device="cuda")
        slots = (bt[:, (ctx - 1) // BS] * BS + (ctx - 1) % BS).contiguous()
        q = torch.randn(B, NQ, D, device="cuda").to(torch.bfloat16)
        out = torch.empty(B, NQ * D, device="cuda", dtype=torch.bfloat16)
        N = (NQ + 2 * NKV) * D
        slab = torch.randn(4 * B * N, device="cuda") * 0.05
        gb = B * ctx * NKV * D * 2 * 2 / 1e9
        # split-partition builds (PK_DECODE_PART < 512) need the partial buffers; q path merges in-launch
        part_o = torch.empty(B * NQ * 8 * D, device="cuda")
        part_ml = torch.empty(B * NQ * 8 * 2, device="cuda")
        ctrs = torch.zeros(B * NKV, dtype=torch.int32, device="cuda")

        def call_q(f, i):
            k, v = layers[i % 4]
            rc = f(out.data_ptr(), q.data_ptr(), k.data_ptr(), v.data_ptr(), bt.data_ptr(), cl.data_ptr(), part_o.data_ptr(),
                   part_ml.data_ptr(), ctrs.data_ptr(), B, NQ, NKV, BS, maxb, NQ * D, NQ * D, 0.088, 512, st())
            assert rc == 0, rc

        def call_qkv(g_, i):
            k, v = layers[i % 4]
            rc = g_(out.data_ptr(), slab.data_ptr(), 4, B, pos.data_ptr(), cs.data_ptr(), slots.data_ptr(),
                    k.data_ptr(), v.data_ptr(), bt.data_ptr(), cl.data_ptr(), part_o.data_ptr(), part_ml.data_ptr(), B, NQ, NKV, BS, maxb,
                    NQ * D, 0.088, 512, st())
            assert rc == 0, rc

        def timeit(fn):
            for i in range(4):
                fn(i)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for i in range(a.iters):
                fn(i)
            e1.record()
            torch.cuda.synchronize()
            return e0.elapsed_time(e1) / a.iters * 1000

        res = {t: {"q": [], "qkv4": []} for t in libs}
        for _ in range(a.rounds):
            for t, (f, g_) in libs.items():
                res[t]["q"].append(timeit(lambda i: call_q(f, i)))
                res[t]["qkv4"].append(timeit(lambda i: call_qkv(g_, i)))
        for t in libs:
            qm, km = statistics.median(res[t]["q"]), statistics.median(res[t]["qkv4"])
            print(json.dumps({"lib": t, "ctx": ctx, "q_us": round(qm, 2), "q_tbs": round(gb / qm * 1e3, 2),
                              "qkv4_us": round(km, 2), "q_min": round(min(res[t]["q"]), 2)}), flush=True)
        del layers


if __name__ == "__main__":
    main()
