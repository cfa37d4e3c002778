"""Weight-streaming decode GEMM (csrc/kernels/gemm_skinny.hip) vs fp32 matmul references."""
import pytest
import torch

from polykey_service_amd.ops import gemm
from polykey_service_amd.ops import reference as ref

pytestmark = pytest.mark.gpu


@pytest.fixture(params=[0, 8], ids=["ring2", "ring4"], autouse=True)
def w_ring_depth(request):
    """Every test runs with the 2-step and the 4-step W register ring (mode bit 3)."""
    old = gemm.DEEP
    gemm.DEEP = request.param
    yield
    gemm.DEEP = old

def rnd(*shape, scale=1.0):
    return (torch.randn(*shape, device="cuda") * scale).to(torch.bfloat16)


@pytest.mark.parametrize("M", [1, 7, 16, 33, 64])
@pytest.mark.parametrize("N,K", [(6144, 4096), (4096, 14336), (1280, 8192), (128256, 4096), (64, 256)])
def test_linear_bf16(M, N, K):
    x, w = rnd(M, K), rnd(N, K, scale=0.02)
    y = gemm.linear(x, w)
    exp = (x.float() @ w.float().t())
    torch.testing.assert_close(y.float(), exp, atol=2e-2, rtol=2e-2)


@pytest.mark.parametrize("M", [3, 64])
@pytest.mark.parametrize("N,K,S", [(4096, 4096, 8), (4096, 14336, 8), (6144, 4096, 4), (512, 1024, 2)])
def test_partial_and_reduce(M, N, K, S):
    x, w = rnd(M, K), rnd(N, K, scale=0.02)
    ws = torch.empty(S * M * N, dtype=torch.float32, device="cuda")
    p = gemm.linear_partial(x, w, ws, S)
    exp = x.float() @ w.float().t()
    torch.testing.assert_close(p.view().sum(0), exp, atol=1e-2, rtol=1e-2)
    torch.testing.assert_close(gemm.reduce_partial(p).float(), exp, atol=2e-2, rtol=2e-2)


@pytest.mark.parametrize("M,I,K", [(5, 14336, 4096), (64, 3584, 8192), (1, 512, 256)])
def test_fused_silu_epilogue(M, I, K):
    x = rnd(M, K)
    g, u = rnd(I, K, scale=0.05), rnd(I, K, scale=0.05)
    w = gemm.interleave_gate_up(g, u)
    exp = ref.silu_and_mul(torch.cat([(x.float() @ g.float().t()), (x.float() @ u.float().t())], -1).to(torch.bfloat16))
    ws = torch.empty(64 * 2 * I * 16, dtype=torch.float32, device="cuda")
    y = gemm.linear_silu(x, w, ws)
    torch.testing.assert_close(y.float(), exp.float(), atol=3e-2, rtol=3e-2)
    # prefill path: hipBLASLt + interleaved SiLU kernel
    y2 = gemm.silu_and_mul_interleaved(torch.nn.functional.linear(x, w))
    torch.testing.assert_close(y2.float(), exp.float(), atol=3e-2, rtol=3e-2)
    g2, u2 = gemm.deinterleave_gate_up(w)
    assert torch.equal(g2, g) and torch.equal(u2, u)


@pytest.mark.parametrize("M,H,S", [(64, 4096, 8), (3, 8192, 4), (17, 1024, 2)])
def test_partial_add_rmsnorm(M, H, S):
    K = 256 * S
    x, w = rnd(M, K), rnd(H, K, scale=0.05)
    res = rnd(M, H)
    nw = rnd(H)
    ws = torch.empty(S * M * H, dtype=torch.float32, device="cuda")
    p = gemm.linear_partial(x, w, ws, S)
    proj = (x.float() @ w.float().t()).to(torch.bfloat16)
    res_ref, x_ref = res.clone().cpu(), proj.clone().cpu()
    ref.fused_add_rms_norm(x_ref, res_ref, nw.cpu(), 1e-5)
    out, res2 = gemm.partial_add_rms_norm(p, res, nw, 1e-5)
    torch.testing.assert_close(res2.cpu().float(), res_ref.float(), atol=3e-2, rtol=2e-2)
    torch.testing.assert_close(out.cpu().float(), x_ref.float(), atol=5e-2, rtol=3e-2)


@pytest.mark.parametrize("nq,nkv,bs,M", [(32, 8, 32, 64), (8, 1, 16, 5)])
def test_qkv_reduce_rope_cache(nq, nkv, bs, M):
    from polykey_service_amd.ops import attention as A
    K, S = 1024, 4
    N = (nq + 2 * nkv) * 128
    x, w = rnd(M, K), rnd(N, K, scale=0.05)
    ws = torch.empty(S * M * N, dtype=torch.float32, device="cuda")
    pos = torch.randint(0, 2000, (M,), dtype=torch.int32, device="cuda")
    cs = ref.rope_cos_sin_cache(2048, 128, 500000.0).cuda()
    nb = M // bs + 4
    slots = torch.randperm(nb * bs, device="cuda")[:M].to(torch.int32)
    slots[0] = -1
    kc = torch.zeros(nb, nkv, bs, 128, dtype=torch.bfloat16, device="cuda")
    vc = torch.zeros(nb, nkv, 128, bs, dtype=torch.bfloat16, device="cuda")
    kc2, vc2 = kc.clone(), vc.clone()
    q = gemm.qkv_reduce_rope_cache(gemm.linear_partial(x, w, ws, S), pos, cs, kc, vc, slots, nq, nkv)
    qkv = (x.float() @ w.float().t()).to(torch.bfloat16)
    A.rope_and_cache(qkv, pos, cs, kc2, vc2, slots, nq, nkv)
    torch.testing.assert_close(q.float(), qkv.view(M, -1, 128)[:, :nq].float(), atol=3e-2, rtol=2e-2)
    torch.testing.assert_close(kc.float(), kc2.float(), atol=3e-2, rtol=2e-2)
    torch.testing.assert_close(vc.float(), vc2.float(), atol=3e-2, rtol=2e-2)


@pytest.mark.parametrize("M", [1, 17, 64])
@pytest.mark.parametrize("N,K,S", [(6144, 4096, 4), (4096, 14336, 8), (128, 256, 1)])
def test_fragment_packed_weights(M, N, K, S):
    x, w = rnd(M, K), rnd(N, K, scale=0.02)
    wp = gemm.pack_weight(w)
    assert torch.equal(gemm.unpack_weight(wp), w)
    exp = x.float() @ w.float().t()
    torch.testing.assert_close(gemm.linear(x, w, packed=wp).float(), exp, atol=2e-2, rtol=2e-2)
    ws = torch.empty(max(S, 1) * M * N, dtype=torch.float32, device="cuda")
    if S > 1:
        p = gemm.linear_partial(x, w, ws, S, packed=wp)
        torch.testing.assert_close(p.view().sum(0), exp, atol=1e-2, rtol=1e-2)


def test_fragment_packed_silu():
    M, I, K = 9, 3584, 4096
    x = rnd(M, K)
    g, u = rnd(I, K, scale=0.05), rnd(I, K, scale=0.05)
    w = gemm.interleave_gate_up(g, u)
    exp = ref.silu_and_mul(torch.cat([(x.float() @ g.float().t()), (x.float() @ u.float().t())], -1).to(torch.bfloat16))
    ws = torch.empty(64 * 2 * I * 16, dtype=torch.float32, device="cuda")
    y = gemm.linear_silu(x, w, ws, packed=gemm.pack_weight(w))
    torch.testing.assert_close(y.float(), exp.float(), atol=3e-2, rtol=3e-2)
