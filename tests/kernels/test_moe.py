"""MoE kernels (csrc/kernels/moe.hip): routing, stable align, grouped GEMM, combine vs fp32 loops."""
import pytest
import torch

from polykey_service_amd.ops import gemm, moe

pytestmark = pytest.mark.gpu


def weights(E, H, I, dev="cuda"):
    g = torch.Generator().manual_seed(0)
    router = (torch.randn(E, H, generator=g) * 0.1).to(torch.bfloat16).to(dev)
    w13 = torch.stack([gemm.interleave_gate_up((torch.randn(I, H, generator=g) * 0.05).to(torch.bfloat16),
                                               (torch.randn(I, H, generator=g) * 0.05).to(torch.bfloat16))
                       for _ in range(E)]).to(dev)
    w2 = (torch.randn(E, H, I, generator=g) * 0.05).to(torch.bfloat16).to(dev)
    return router, w13, w2


def test_topk_softmax():
    g = torch.Generator().manual_seed(0)
    x = torch.randn(100, 8, generator=g).to(torch.bfloat16)
    x[0, 3] = x[0, 5] = 4.0  # exact tie: the kernel picks the lower expert id
    x = x.cuda()
    ids, w = moe.topk_softmax(x, 2)
    p = torch.softmax(x.float(), -1)
    ew, eids = torch.sort(p, dim=-1, descending=True, stable=True)
    ew, eids = ew[:, :2], eids[:, :2]
    assert torch.equal(ids.long().cpu(), eids.cpu())
    torch.testing.assert_close(w.cpu(), (ew / ew.sum(-1, keepdim=True)).cpu(), atol=1e-5, rtol=1e-5)


@pytest.mark.parametrize("n,E,lo,hi", [(2, 8, 0, 8), (128, 8, 0, 8), (5000, 8, 2, 4), (3000, 64, 0, 64)])
def test_align_stable_matches_cpu(n, E, lo, hi):
    ids = torch.randint(0, E, (n,), dtype=torch.int32)
    off_c, s_c, inv_c = moe.align(ids, E, lo, hi)
    off_g, s_g, inv_g = moe.align(ids.cuda(), E, lo, hi)
    m = int(off_c[-1])
    assert torch.equal(off_g.cpu(), off_c)
    assert torch.equal(s_g.cpu()[:m], s_c)
    assert torch.equal(inv_g.cpu(), inv_c)


@pytest.mark.parametrize("T", [1, 7, 64, 300])
@pytest.mark.parametrize("ep", [(0, 8), (2, 4)])
def test_fused_moe(T, ep):
    E, H, I = 8, 512, 1024
    router, w13, w2 = weights(E, H, I)
    lo, hi = ep
    x = torch.randn(T, H, device="cuda").to(torch.bfloat16)
    y = moe.fused_moe(x, router, w13[lo:hi].contiguous(), w2[lo:hi].contiguous(), 2, lo, hi)
    ref = moe.fused_moe_reference(x, router, w13[lo:hi], w2[lo:hi], 2, lo, hi)
    torch.testing.assert_close(y.float(), ref, atol=3e-2, rtol=3e-2)


@pytest.mark.parametrize("T", [1, 9, 64])
def test_fused_moe_packed_experts(T):
    """Decode MoE through the grouped weight-streaming GEMM with fragment-packed experts."""
    E, H, I = 8, 512, 1024
    router, w13, w2 = weights(E, H, I)
    x = torch.randn(T, H, device="cuda").to(torch.bfloat16)
    w13_p = gemm.pack_weight(w13.view(-1, H)).view(w13.shape)
    w2_p = gemm.pack_weight(w2.view(-1, I)).view(w2.shape)
    y = moe.fused_moe(x, router, w13, w2, 2, 0, E, w13_p, w2_p)
    ref = moe.fused_moe_reference(x, router, w13, w2, 2, 0, E)
    torch.testing.assert_close(y.float(), ref, atol=3e-2, rtol=3e-2)


def test_grouped_linear_skips_empty_groups_and_splits():
    G, N, K, R = 4, 256, 512, 40
    a = torch.randn(R, K, device="cuda").to(torch.bfloat16)
    w = (torch.randn(G, N, K, device="cuda") * 0.05).to(torch.bfloat16)
    offsets = torch.tensor([0, 17, 17, 40, 40], dtype=torch.int32, device="cuda")  # groups 1 and 3 empty
    y = gemm.grouped_linear(a, w, offsets, 23, silu=False)
    exp = torch.cat([a[:17].float() @ w[0].float().t(), a[17:40].float() @ w[2].float().t()])
    torch.testing.assert_close(y.float(), exp, atol=2e-2, rtol=2e-2)
    ws = torch.empty(2 * R * N, dtype=torch.float32, device="cuda")
    p = gemm.grouped_linear(a, w, offsets, 23, silu=False, packed=gemm.pack_weight(w.view(-1, K)).view(w.shape),
                            ws=ws, S=2)
    torch.testing.assert_close(p[: 2 * R * N].view(2, R, N).sum(0), exp, atol=2e-2, rtol=2e-2)


@pytest.mark.parametrize("bound", [128, 256, 512])
def test_grouped_linear_row_tiles(bound):
    """Expert groups above 64 rows (EP: every sender's tokens can pick one expert): 128-row tiles
    per group, bf16 out, packed SiLU and split-K slabs; empty groups read nothing."""
    G, N, K = 4, 512, 1024
    sizes = [min(bound, s) for s in (130, 0, 64, 200)]
    offs = [0]
    for n in sizes:
        offs.append(offs[-1] + n)
    R = offs[-1]
    a = torch.randn(R, K, device="cuda").to(torch.bfloat16)
    w = (torch.randn(G, N, K, device="cuda") * 0.05).to(torch.bfloat16)
    offsets = torch.tensor(offs, dtype=torch.int32, device="cuda")
    exp = torch.cat([a[offs[e]:offs[e + 1]].float() @ w[e].float().t() for e in range(G)])
    y = gemm.grouped_linear(a, w, offsets, bound, silu=False)
    torch.testing.assert_close(y.float(), exp, atol=2e-2, rtol=2e-2)
    wp = gemm.pack_weight(w.view(-1, K)).view(w.shape)
    ws = torch.empty(2 * R * N, dtype=torch.float32, device="cuda")
    p = gemm.grouped_linear(a, w, offsets, bound, silu=False, packed=wp, ws=ws, S=2)
    torch.testing.assert_close(p[: 2 * R * N].view(2, R, N).sum(0), exp, atol=2e-2, rtol=2e-2)
    h = gemm.grouped_linear(a, w, offsets, bound, silu=True, packed=wp)
    from polykey_service_amd.ops import reference as ref
    torch.testing.assert_close(h.float(), ref.silu_and_mul_interleaved(exp.to(torch.bfloat16)).float(),
                               atol=3e-2, rtol=3e-2)


@pytest.mark.parametrize("M,E,k", [(1, 8, 2), (64, 8, 2), (17, 64, 4)])
def test_add_rmsnorm_with_routing(M, E, k):
    """Split-K residual add + RMSNorm that also routes each row == norm kernel + router GEMM
    (bf16 logits) + topk_softmax."""
    from polykey_service_amd.ops import gemm
    H, S = 4096, 4
    g = torch.Generator().manual_seed(M + E)
    slabs = (torch.randn(S, M, H, generator=g) * 0.3).cuda()
    res = torch.randn(M, H, generator=g).to(torch.bfloat16).cuda()
    nw = (1 + 0.1 * torch.randn(H, generator=g)).to(torch.bfloat16).cuda()
    router = (torch.randn(E, H, generator=g) * 0.05).to(torch.bfloat16).cuda()
    ws = slabs.reshape(-1).clone()
    p = gemm.Partial(ws, S, M, H)
    x1, r1 = gemm.partial_add_rms_norm(p, res.clone(), nw, 1e-5)
    x2, r2, ids, w = gemm.partial_add_rms_norm_route(p, res.clone(), nw, 1e-5, router, k)
    assert torch.equal(x1, x2) and torch.equal(r1, r2)
    ids_ref, w_ref = moe.topk_softmax(torch.nn.functional.linear(x1, router), k)
    logits = torch.nn.functional.linear(x1, router).float()
    top = logits.topk(min(k + 1, E), -1).values
    clear = ((top[:, :-1] - top[:, 1:]).abs() > 1e-2).all(-1)  # rows without a bf16 near-tie
    assert torch.equal(ids[clear], ids_ref[clear])
    torch.testing.assert_close(w[clear], w_ref[clear], atol=2e-2, rtol=2e-2)


@pytest.mark.parametrize("T,ep", [(5, (0, 8)), (64, (0, 8)), (33, (2, 6))])
def test_decode_moe_gather_and_fused_combine(T, ep):
    """Decode MoE (routing kernel, gathered-A w13 GEMM, deferred combine fused with the residual
    add + RMSNorm) vs the fp32 reference followed by add + RMSNorm."""
    from polykey_service_amd.ops import reference as ref
    E, H, I = 8, 1024, 1024
    router, w13, w2 = weights(E, H, I)
    lo, hi = ep
    x = torch.randn(T, H, device="cuda").to(torch.bfloat16)
    res = torch.randn(T, H, device="cuda").to(torch.bfloat16)
    nw = (1 + 0.1 * torch.randn(H, device="cuda")).to(torch.bfloat16)
    pend = moe.fused_moe(x, router, w13[lo:hi].contiguous(), w2[lo:hi].contiguous(), 2, lo, hi, defer_combine=True)
    assert isinstance(pend, moe.PendingCombine)
    y_ref = moe.fused_moe_reference(x, router, w13[lo:hi], w2[lo:hi], 2, lo, hi)
    torch.testing.assert_close(pend.combine().float(), y_ref, atol=3e-2, rtol=3e-2)
    r1 = res.clone()
    xo, r1 = moe.combine_add_rms_norm(pend, r1, nw, 1e-5)
    r_ref = (pend.combine().float() + res.float()).to(torch.bfloat16)
    torch.testing.assert_close(r1.float(), r_ref.float(), atol=3e-2, rtol=2e-2)
    torch.testing.assert_close(xo.float(), ref.rms_norm(r_ref, nw, 1e-5).float(), atol=5e-2, rtol=3e-2)
