"""Paged decode / prefill attention and fused RoPE+cache kernels vs fp32 references."""
import math

import pytest
import torch

from polykey_service_amd.ops import attention as A
from polykey_service_amd.ops import reference as ref

pytestmark = pytest.mark.gpu
HD = 128


def make_cache(num_blocks, nkv, bs, seed=0):
    g = torch.Generator().manual_seed(seed)
    k = torch.randn(num_blocks, nkv, bs, HD, generator=g).to(torch.bfloat16)
    v = torch.randn(num_blocks, nkv, HD, bs, generator=g).to(torch.bfloat16)
    return k, v


def block_tables_for(ctxs, bs, num_blocks, max_blocks, seed=0):
    g = torch.Generator().manual_seed(seed + 7)
    perm = torch.randperm(num_blocks, generator=g).tolist()
    bt = torch.zeros(len(ctxs), max_blocks, dtype=torch.int32)
    i = 0
    for s, c in enumerate(ctxs):
        nb = (c + bs - 1) // bs
        bt[s, :nb] = torch.tensor(perm[i:i + nb], dtype=torch.int32)
        i += nb
    return bt


@pytest.mark.parametrize("nq,nkv,bs", [(32, 8, 32), (8, 1, 32), (32, 8, 96), (4, 4, 32), (16, 1, 64)])
@pytest.mark.parametrize("ctxs", [[1, 5, 32, 33, 100], [512, 513, 1200, 7], [2048, 1], [5000, 3, 2600]])
def test_decode(nq, nkv, bs, ctxs):
    max_blocks = (max(ctxs) + bs - 1) // bs + 3
    nb = sum((c + bs - 1) // bs for c in ctxs) + 4
    kc, vc = make_cache(nb, nkv, bs)
    bt = block_tables_for(ctxs, bs, nb, max_blocks)
    B = len(ctxs)
    qkv = torch.randn(B, (nq + 2 * nkv) * HD).to(torch.bfloat16)
    q = qkv.view(B, nq + 2 * nkv, HD)[:, :nq]
    cl = torch.tensor(ctxs, dtype=torch.int32)
    scale = 1 / math.sqrt(HD)
    exp = ref.paged_attention(q.contiguous(), kc, vc, bt, cl, torch.arange(B + 1, dtype=torch.int32), scale)
    d = "cuda"
    qkv_d = qkv.to(d)
    q_d = qkv_d.view(B, nq + 2 * nkv, HD)[:, :nq]
    po, pml = A.decode_workspace(B, nq, max_blocks, bs, d)
    md = A.AttnMetadata(num_decode=B, num_prefill=0, num_prefill_tokens=0, max_prefill_q_len=0,
                        slot_mapping=torch.zeros(B, dtype=torch.int32, device=d),
                        decode_block_tables=bt.to(d), decode_context_lens=cl.to(d), decode_part_o=po,
                        decode_part_ml=pml)
    kcd, vcd = kc.to(d), vc.to(d)
    for _ in range(2):  # repeated launches reuse the partition slabs
        out = A.paged_attention(q_d, kcd, vcd, md, scale)
        torch.testing.assert_close(out.cpu().view(B, nq, HD).float(), exp.float(), atol=2e-2, rtol=2e-2)


def test_decode_zero_context_rows_are_zero():
    nq, nkv, bs = 8, 2, 32
    kc, vc = make_cache(8, nkv, bs)
    bt = torch.zeros(3, 4, dtype=torch.int32)
    cl = torch.tensor([0, 40, 0], dtype=torch.int32)
    bt[1, :2] = torch.tensor([3, 5])
    q = torch.randn(3, nq, HD).to(torch.bfloat16)
    md = A.AttnMetadata(3, 0, 0, 0, torch.zeros(3, dtype=torch.int32, device="cuda"), bt.cuda(), cl.cuda())
    out = A.paged_attention(q.cuda(), kc.cuda(), vc.cuda(), md, 0.1).cpu().view(3, nq, HD)
    assert torch.all(out[0] == 0) and torch.all(out[2] == 0)
    exp = ref.paged_attention(q[1:2], kc, vc, bt[1:2], cl[1:2], torch.tensor([0, 1], dtype=torch.int32), 0.1)
    torch.testing.assert_close(out[1:2].float(), exp.float(), atol=2e-2, rtol=2e-2)


@pytest.mark.parametrize("nq,nkv,bs", [(32, 8, 32), (8, 1, 32), (4, 1, 64), (16, 1, 32), (64, 8, 32)])
@pytest.mark.parametrize("qlens,ctxs", [([7, 16, 33], [7, 16, 33]), ([1, 20, 64], [100, 20, 300]),
                                        ([130], [130]), ([5, 1], [70, 1]), ([300, 77], [1000, 77])])
def test_prefill_with_prefix(nq, nkv, bs, qlens, ctxs):
    max_blocks = (max(ctxs) + bs - 1) // bs
    nb = sum((c + bs - 1) // bs for c in ctxs) + 2
    kc, vc = make_cache(nb, nkv, bs, seed=3)
    bt = block_tables_for(ctxs, bs, nb, max_blocks, seed=3)
    T = sum(qlens)
    qkv = torch.randn(T, (nq + 2 * nkv) * HD).to(torch.bfloat16)
    q = qkv.view(T, nq + 2 * nkv, HD)[:, :nq]
    cu = torch.tensor([0] + list(torch.cumsum(torch.tensor(qlens), 0)), dtype=torch.int32)
    cl = torch.tensor(ctxs, dtype=torch.int32)
    scale = 1 / math.sqrt(HD)
    exp = ref.paged_attention(q.contiguous(), kc, vc, bt, cl, cu, scale)
    d = "cuda"
    md = A.AttnMetadata(0, len(qlens), T, max(qlens), torch.zeros(T, dtype=torch.int32, device=d),
                        prefill_block_tables=bt.to(d), prefill_context_lens=cl.to(d), prefill_cu_q=cu.to(d))
    qkv_d = qkv.to(d)
    out = A.paged_attention(qkv_d.view(T, nq + 2 * nkv, HD)[:, :nq], kc.to(d), vc.to(d), md, scale)
    torch.testing.assert_close(out.cpu().view(T, nq, HD).float(), exp.float(), atol=2e-2, rtol=2e-2)


def test_mixed_decode_and_prefill():
    nq, nkv, bs = 16, 4, 32
    dctx, qlens, pctx = [40, 600], [9, 30], [9, 75]
    ctxs = dctx + pctx
    max_blocks = 24
    nb = 64
    kc, vc = make_cache(nb, nkv, bs, seed=5)
    bt = block_tables_for(ctxs, bs, nb, max_blocks, seed=5)
    T = 2 + sum(qlens)
    q = torch.randn(T, nq, HD).to(torch.bfloat16)
    scale = 0.09
    cu = torch.tensor([0, 9, 39], dtype=torch.int32)
    exp_d = ref.paged_attention(q[:2], kc, vc, bt[:2], torch.tensor(dctx), torch.arange(3, dtype=torch.int32), scale)
    exp_p = ref.paged_attention(q[2:], kc, vc, bt[2:], torch.tensor(pctx), cu, scale)
    d = "cuda"
    po, pml = A.decode_workspace(2, nq, max_blocks, bs, d)
    md = A.AttnMetadata(2, 2, sum(qlens), 30, torch.zeros(T, dtype=torch.int32, device=d),
                        bt[:2].to(d), torch.tensor(dctx, dtype=torch.int32, device=d), bt[2:].to(d),
                        torch.tensor(pctx, dtype=torch.int32, device=d), cu.to(d), po, pml)
    out = A.paged_attention(q.to(d), kc.to(d), vc.to(d), md, scale).cpu().view(T, nq, HD)
    torch.testing.assert_close(out[:2].float(), exp_d.float(), atol=2e-2, rtol=2e-2)
    torch.testing.assert_close(out[2:].float(), exp_p.float(), atol=2e-2, rtol=2e-2)


@pytest.mark.parametrize("nq,nkv,bs", [(32, 8, 32), (8, 1, 96), (4, 2, 64)])
def test_rope_and_cache(nq, nkv, bs):
    T = 37
    qkv = torch.randn(T, (nq + 2 * nkv) * HD).to(torch.bfloat16)
    pos = torch.randint(0, 4000, (T,), dtype=torch.int32)
    cs = ref.rope_cos_sin_cache(4096, HD, 500000.0)
    nb = 8 + T // bs * 2
    slots = torch.randperm(nb * bs)[:T].to(torch.int32)
    slots[3] = -1
    kc = torch.zeros(nb, nkv, bs, HD, dtype=torch.bfloat16)
    vc = torch.zeros(nb, nkv, HD, bs, dtype=torch.bfloat16)
    qkv_r, kc_r, vc_r = qkv.clone(), kc.clone(), vc.clone()
    ref.rope_and_cache(qkv_r, pos, cs, kc_r, vc_r, slots, nq, nkv, HD)
    d = "cuda"
    qkv_d, kc_d, vc_d = qkv.to(d), kc.to(d), vc.to(d)
    A.rope_and_cache(qkv_d, pos.to(d), cs.to(d), kc_d, vc_d, slots.to(d), nq, nkv, HD)
    torch.testing.assert_close(qkv_d.cpu().float(), qkv_r.float(), atol=1.6e-2, rtol=1e-2)
    torch.testing.assert_close(kc_d.cpu().float(), kc_r.float(), atol=1.6e-2, rtol=1e-2)
    assert torch.equal(vc_d.cpu(), vc_r)


@pytest.mark.parametrize("nq,nkv,bs", [(32, 8, 32), (8, 2, 64)])
def test_rope_and_cache_aligned_runs(nq, nkv, bs):
    """Prefill layout: 32-token groups that fill an aligned 32-slot run of a block take the
    transposed V-tile path; a misaligned group, a group with a padding row and a short tail
    take the per-token path -- both bit-exact against the reference."""
    nb = 12
    runs = [list(range(2 * bs, 2 * bs + 32)),               # aligned, block 2
            list(range(5 * bs + bs - 32, 5 * bs + bs)),     # aligned, last 32 slots of block 5
            list(range(7 * bs + 3, 7 * bs + 35)),           # misaligned start
            list(range(9 * bs, 9 * bs + 32)),               # aligned but one padding row
            list(range(11 * bs, 11 * bs + 5))]              # tail of 5 tokens
    runs[3][7] = -1
    slots = torch.tensor(sum(runs, []), dtype=torch.int32)
    T = slots.numel()
    qkv = torch.randn(T, (nq + 2 * nkv) * HD).to(torch.bfloat16)
    pos = torch.arange(T, dtype=torch.int32)
    cs = ref.rope_cos_sin_cache(4096, HD, 500000.0)
    kc = torch.zeros(nb, nkv, bs, HD, dtype=torch.bfloat16)
    vc = torch.zeros(nb, nkv, HD, bs, dtype=torch.bfloat16)
    qkv_r, kc_r, vc_r = qkv.clone(), kc.clone(), vc.clone()
    ref.rope_and_cache(qkv_r, pos, cs, kc_r, vc_r, slots, nq, nkv, HD)
    d = "cuda"
    qkv_d, kc_d, vc_d = qkv.to(d), kc.to(d), vc.to(d)
    A.rope_and_cache(qkv_d, pos.to(d), cs.to(d), kc_d, vc_d, slots.to(d), nq, nkv, HD)
    torch.testing.assert_close(qkv_d.cpu().float(), qkv_r.float(), atol=1.6e-2, rtol=1e-2)
    torch.testing.assert_close(kc_d.cpu().float(), kc_r.float(), atol=1.6e-2, rtol=1e-2)
    assert torch.equal(vc_d.cpu(), vc_r)


@pytest.mark.parametrize("nq,nkv,bs", [(32, 8, 32), (8, 1, 64), (16, 4, 32)])
@pytest.mark.parametrize("ctxs", [[1, 5, 33, 300], [512, 513, 1300, 0]])
@pytest.mark.parametrize("S", [1, 4])
@pytest.mark.parametrize("pos_last", [True, False])
def test_decode_from_qkv_slabs(nq, nkv, bs, ctxs, S, pos_last):
    """Attention kernel fed by the QKV split-K slabs (reduce + RoPE + cache write folded in) vs
    the unfused kernels: same output, same K/V cache contents; ctx 0 = padded row (slot -1).
    pos_last: the new token's position is ctx - 1 (its key is folded in from LDS and the cache
    row stored at the end); otherwise the kernel writes the row first and attends through the cache."""
    from polykey_service_amd.ops import gemm
    d = "cuda"
    B = len(ctxs)
    N = (nq + 2 * nkv) * HD
    max_blocks = (max(ctxs) + bs - 1) // bs + 3
    nb = sum((max(c, 1) + bs - 1) // bs for c in ctxs) + 4
    kc, vc = make_cache(nb, nkv, bs, seed=3)
    bt = block_tables_for([max(c, 1) for c in ctxs], bs, nb, max_blocks, seed=3)
    cl = torch.tensor(ctxs, dtype=torch.int32)
    pos = (cl - 1).clamp(min=0) if pos_last else (cl // 2).clamp(min=0)
    slots = torch.tensor([int(bt[i, (c - 1) // bs]) * bs + (c - 1) % bs if c > 0 else -1 for i, c in enumerate(ctxs)],
                         dtype=torch.int32)
    g = torch.Generator().manual_seed(5)
    slabs = (torch.randn(S, B, N, generator=g) * (0.5 / S)).to(d)
    cs = ref.rope_cos_sin_cache(4096, HD, 500000.0).to(d)
    ws = torch.empty(S * B * N, dtype=torch.float32, device=d)
    ws[: S * B * N].copy_(slabs.reshape(-1))
    p = gemm.Partial(ws, S, B, N)
    po, pml = A.decode_workspace(B, nq, max_blocks, bs, d)
    mk = lambda: A.AttnMetadata(num_decode=B, num_prefill=0, num_prefill_tokens=0, max_prefill_q_len=0,
                                slot_mapping=slots.to(d), decode_block_tables=bt.to(d), decode_context_lens=cl.to(d),
                                decode_part_o=po, decode_part_ml=pml)
    scale = 1 / math.sqrt(HD)
    k1, v1 = kc.to(d), vc.to(d)
    q = gemm.qkv_reduce_rope_cache(p, pos.to(d), cs, k1, v1, slots.to(d), nq, nkv)
    exp = A.paged_attention(q, k1, v1, mk(), scale)
    k2, v2 = kc.to(d), vc.to(d)
    got = A.paged_decode_from_qkv(p, pos.to(d), cs, k2, v2, mk(), scale, nq, nkv)
    torch.testing.assert_close(got.float(), exp.float(), atol=2e-2, rtol=2e-2)
    assert torch.equal(k1, k2) and torch.equal(v1, v2)


@pytest.mark.parametrize("nq,nkv,bs,H", [(32, 8, 32, 1024), (16, 4, 32, 1024), (64, 8, 32, 1024),
                                         (32, 8, 32, 4096), (8, 1, 32, 8192)])
@pytest.mark.parametrize("ctxs", [[1, 5, 33, 300], [384] * 64, [512, 513, 1300, 0], [40 + 3 * i for i in range(100)]])
@pytest.mark.parametrize("pos_last", [True, False])
def test_qkv_attn_fused_matches_two_launches(nq, nkv, bs, H, ctxs, pos_last):
    """Fused QKV projection -> decode attention launch (csrc/kernels/decode_fused.hip): the QKV
    tiles hand their write-through slabs to the attention tiles in-launch.  Attention output and
    K / V cache bit-identical to linear_partial_rowscale + paged_decode_from_qkv, over repeated
    launches with new inputs (stale slabs would show), tickets left zeroed."""
    from polykey_service_amd.ops import gemm
    d = "cuda"
    B = len(ctxs)  # H: 8B width (32 q / 8 kv heads) and the 70B TP=8 shard (8 q / 1 kv head, H 8192)
    N = (nq + 2 * nkv) * HD
    max_blocks = (max(ctxs) + bs - 1) // bs + 3
    nb = sum((max(c, 1) + bs - 1) // bs for c in ctxs) + 4
    bt = block_tables_for([max(c, 1) for c in ctxs], bs, nb, max_blocks, seed=3)
    cl = torch.tensor(ctxs, dtype=torch.int32)
    # pos_last False: the new token is not the last key (the writer stores it before attending,
    # no K/V prefetch for that workgroup)
    pos = (cl - 1).clamp(min=0) if pos_last else (cl // 2).clamp(min=0)
    slots = torch.tensor([int(bt[i, (c - 1) // bs]) * bs + (c - 1) % bs if c > 0 else -1 for i, c in enumerate(ctxs)],
                         dtype=torch.int32)
    cs = ref.rope_cos_sin_cache(4096, HD, 500000.0).to(d)
    po, pml = A.decode_workspace(B, nq, max_blocks, bs, d)
    mk = lambda: A.AttnMetadata(num_decode=B, num_prefill=0, num_prefill_tokens=0, max_prefill_q_len=0,
                                slot_mapping=slots.to(d), decode_block_tables=bt.to(d), decode_context_lens=cl.to(d),
                                decode_part_o=po, decode_part_ml=pml)
    scale = 1 / math.sqrt(HD)
    w = (torch.randn(N, H, device=d) * 0.05).to(torch.bfloat16)
    wp = gemm.pack_weight(w)
    S = gemm.choose_split(N, H, B)
    ws1 = torch.empty(S * B * N, dtype=torch.float32, device=d)
    ws2 = torch.empty_like(ws1)
    flow = torch.zeros(gemm.FLOW_WORDS, dtype=torch.int32, device=d)
    kc, vc = make_cache(nb, nkv, bs, seed=3)
    k1, v1, k2, v2 = kc.to(d), vc.to(d), kc.to(d), vc.to(d)
    for it in range(4):
        res = (torch.randn(B, H, device=d)).to(torch.bfloat16)
        parts = gemm.residual_parts(None, res.clone(), torch.empty((H // gemm.PART_COLS) * B, device=d))
        rs = gemm.RowScale(parts, 1e-5)
        p = gemm.linear_partial_rowscale(res, w, ws1, rs, S=S, packed=wp)
        exp = A.paged_decode_from_qkv(p, pos.to(d), cs, k1, v1, mk(), scale, nq, nkv)
        ws2.fill_(float("nan"))
        got = gemm.qkv_attn_fused(res, wp, rs, ws2, pos.to(d), cs, k2, v2, mk(), scale, nq, nkv, flow)
        torch.testing.assert_close(got, exp, atol=0, rtol=0)
        assert torch.equal(k1, k2) and torch.equal(v1, v2)
    torch.cuda.synchronize()
    assert int(flow.abs().sum()) == 0, flow.nonzero().tolist()
