"""Decode attention of the Llama-3-70B TP=8 shard in isolation (8 q / 1 kv head per rank, 64
sequences): where do its ~11 us go?  Each variant is captured as a graph of 80 back-to-back
launches over 80 layers' KV caches (cold, like a decode step) and reported in us per launch:

  qkv S=16 / 8 / 1   attention fed from the QKV projection's split-K slabs (the serving chain)
  q                  q given in bf16 (no slab reduction / RoPE / cache write)
  ctx 32             one 32-key step per sequence: the launch's fixed cost
  fill 0             512-key partitions (64 workgroups, no merge launch) instead of 128-key ones
  wide               8-wave workgroups (launches of <= 128 workgroups)
  merge              partitions merged in-launch by the last to arrive (no reduce launch)

    python tools/attn70_probe.py [--ctx 384] [--batch 64] [--heads 8,1]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from polykey_service_amd.ops import attention as A  # noqa: E402
from polykey_service_amd.ops import gemm, native  # noqa: E402
from polykey_service_amd.ops import reference as ref  # noqa: E402

HD, BS, L = 128, 32, 80
NQ, NKV = 8, 1  # --heads


def run(B, ctx, S, mode, iters=10, merge=False):
    dev = "cuda"
    maxb = (max(ctx, 512) + BS) // BS + 1
    nblk = B * maxb + 1
    kv = [(torch.randn(nblk, NKV, BS, HD, device=dev).to(torch.bfloat16),
           torch.randn(nblk, NKV, HD, BS, device=dev).to(torch.bfloat16)) for _ in range(L)]
    bt = torch.arange(B * maxb, dtype=torch.int32, device=dev).view(B, maxb)
    cl = torch.full((B,), ctx, dtype=torch.int32, device=dev)
    pos = cl - 1
    slots = (bt[:, (ctx - 1) // BS] * BS + (ctx - 1) % BS).to(torch.int32)
    cs = ref.rope_cos_sin_cache(4096, HD, 500000.0).to(dev)
    po, pml = A.decode_workspace(B, NQ, maxb, BS, dev)  # sized for any partition choice
    N = (NQ + 2 * NKV) * HD
    p = gemm.Partial(torch.randn(S * B * N, device=dev) * 0.1, S, B, N)
    q = torch.randn(B, N, device=dev).to(torch.bfloat16).view(B, NQ + 2 * NKV, HD)[:, :NQ]
    md = A.AttnMetadata(num_decode=B, num_prefill=0, num_prefill_tokens=0, max_prefill_q_len=0, slot_mapping=slots,
                        decode_block_tables=bt, decode_context_lens=cl, decode_part_o=po, decode_part_ml=pml,
                        decode_max_ctx=512,
                        decode_counters=torch.zeros((B, NKV), dtype=torch.int32, device=dev) if merge else None)
    scale = HD ** -0.5

    def step():
        for i in range(L):
            if mode == "q":
                A.paged_attention(q, kv[i][0], kv[i][1], md, scale)
            else:
                A.paged_decode_from_qkv(p, pos, cs, kv[i][0], kv[i][1], md, scale, NQ, NKV)

    step()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        step()
    torch.cuda.current_stream().wait_stream(s)
    with torch.cuda.graph(g):
        step()
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        g.replay()
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) / iters / L * 1000
    del g, kv
    return round(us, 2)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ctx", type=int, default=384)
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--heads", default="8,1", help="q,kv heads per rank (8B TP=1: 32,8)")
    a = ap.parse_args()
    global NQ, NKV
    NQ, NKV = (int(x) for x in a.heads.split(","))
    A.apply_decode_fill()
    kv_mb = a.batch * a.ctx * NKV * HD * 2 * 2 / 1e6
    rows = []
    for name, S, mode, ctx, fill, wide, merge in (("qkv S16", 16, "qkv", a.ctx, 256, 0, 0),
                                                  ("qkv S16 merge", 16, "qkv", a.ctx, 256, 0, 1),
                                                  ("qkv S16 fill0", 16, "qkv", a.ctx, 0, 0, 0),
                                                  ("qkv S16 fill0 wide", 16, "qkv", a.ctx, 0, 1, 0),
                                                  ("qkv S8 fill0", 8, "qkv", a.ctx, 0, 0, 0),
                                                  ("qkv S8 fill0 wide", 8, "qkv", a.ctx, 0, 1, 0),
                                                  ("qkv S4", 4, "qkv", a.ctx, 256, 0, 0),
                                                  ("q", 1, "q", a.ctx, 256, 0, 0), ("q fill0", 1, "q", a.ctx, 0, 0, 0),
                                                  ("qkv S16 ctx32", 16, "qkv", 32, 256, 0, 0),
                                                  ("q ctx32", 1, "q", 32, 256, 0, 0)):
        native.call("pk_set_decode_fill", fill)
        native.call("pk_set_decode_wide", wide)
        us = run(a.batch, ctx, S, mode, merge=bool(merge))
        rows.append({"heads": a.heads, "variant": name, "ctx": ctx, "us": us, "kv_tbs": round(kv_mb * ctx / a.ctx / us, 2)})
        print(json.dumps(rows[-1]), flush=True)
    native.call("pk_set_decode_fill", 256)
    native.call("pk_set_decode_wide", 0)


if __name__ == "__main__":
    main()
