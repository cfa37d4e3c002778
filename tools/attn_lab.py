"""Decode attention at the headline bench shape (Llama-3-8B: 32 q / 8 kv heads, d 128, block 32,
64 sequences), rotating over 4 layers' KV caches like a real decode step:

    python tools/attn_lab.py [--ctx 256,384,512] [--iters 40]

Times (us per call, TB/s of K/V bytes):
  q      : pk_paged_decode with q given (short-context launch: one partition)
  qkv S  : pk_paged_decode_qkv from S fp32 QKV slabs (the engine's fused decode path: slab
           reduce + RoPE + KV-cache write in the prologue, then attention)
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from polykey_service_amd.ops import reference  # noqa: E402
from polykey_service_amd.ops import attention as A  # noqa: E402
from polykey_service_amd.ops import gemm  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ctx", default="256,384,512")
    ap.add_argument("--iters", type=int, default=40)
    ap.add_argument("--tag", default="")
    ap.add_argument("--bs", type=int, default=32)
    ap.add_argument("--seq-blocks", action="store_true", help="sequential block tables (else random)")
    a = ap.parse_args()
    B, NQ, NKV, D, BS = 64, 32, 8, 128, a.bs
    cs = reference.rope_cos_sin_cache(8192, 128, 500000.0, None, device="cuda")
    for ctx in (int(c) for c in a.ctx.split(",")):
        maxb = 16384 // BS
        nblk = B * ((ctx + BS) // BS) + 8
        g = torch.Generator(device="cuda").manual_seed(0)
        layers = [(torch.randn(nblk, NKV, BS, D, device="cuda", generator=g).to(torch.bfloat16),
                   torch.randn(nblk, NKV, D, BS, device="cuda", generator=g).to(torch.bfloat16)) for _ in range(4)]
        per = (ctx + BS) // BS
        perm = (torch.arange(B * per) if a.seq_blocks else
                torch.randperm(B * per, generator=torch.Generator().manual_seed(1))).to(torch.int32)
        bt = torch.zeros((B, maxb), dtype=torch.int32)
        bt[:, :per] = perm.view(B, per)
        bt = bt.cuda()
        cl = torch.full((B,), ctx, dtype=torch.int32, device="cuda")
        pos = torch.full((B,), ctx - 1, dtype=torch.int32, device="cuda")
        slots = (bt[:, (ctx - 1) // BS] * BS + (ctx - 1) % BS).contiguous()
        q = torch.randn(B, NQ, D, device="cuda").to(torch.bfloat16)
        md = A.AttnMetadata(num_decode=B, num_prefill=0, num_prefill_tokens=0, max_prefill_q_len=0,
                            slot_mapping=slots, decode_block_tables=bt, decode_context_lens=cl, decode_max_ctx=512)
        N = (NQ + 2 * NKV) * D
        res = {"tag": a.tag, "ctx": ctx, "bs": BS, "seq_blocks": a.seq_blocks}
        gb = B * ctx * NKV * D * 2 * 2 / 1e9

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

        us = timeit(lambda i: A.paged_attention(q, *layers[i % 4], md, 0.088))
        res["q_us"] = round(us, 2)
        res["q_tbs"] = round(gb / us * 1e3, 2)
        for S in (2, 4):
            buf = torch.randn(S * B * N, device="cuda") * 0.05
            p = gemm.Partial(buf, S, B, N)
            us = timeit(lambda i: A.paged_decode_from_qkv(p, pos, cs, *layers[i % 4], md, 0.088, NQ, NKV))
            res[f"qkv{S}_us"] = round(us, 2)
        print(json.dumps(res), flush=True)
        del layers


if __name__ == "__main__":
    main()
