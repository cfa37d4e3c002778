"""RMSNorm / fused-add RMSNorm / SiLU-mul HIP kernels vs fp32 PyTorch references."""
import pytest
import torch

from polykey_service_amd import ops
from polykey_service_amd.ops import reference as ref

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("T,H", [(1, 512), (7, 4096), (64, 4096), (33, 8192), (3, 1024), (5, 2048)])
def test_rmsnorm(T, H):
    torch.manual_seed(0)
    x = torch.randn(T, H, device="cuda", dtype=torch.bfloat16) * 3
    w = torch.randn(H, device="cuda", dtype=torch.bfloat16)
    y = ops.rms_norm(x, w, 1e-5)
    torch.cuda.synchronize()
    r = ref.rms_norm(x.cpu(), w.cpu(), 1e-5)
    torch.testing.assert_close(y.cpu().float(), r.float(), atol=2e-2, rtol=1.6e-2)


@pytest.mark.parametrize("T,H", [(1, 512), (64, 4096), (17, 8192)])
def test_fused_add_rmsnorm(T, H):
    torch.manual_seed(1)
    x = torch.randn(T, H, device="cuda", dtype=torch.bfloat16)
    res = torch.randn(T, H, device="cuda", dtype=torch.bfloat16)
    w = torch.randn(H, device="cuda", dtype=torch.bfloat16)
    xr, rr = x.cpu().clone(), res.cpu().clone()
    ops.fused_add_rms_norm(x, res, w, 1e-5)
    ref.fused_add_rms_norm(xr, rr, w.cpu(), 1e-5)
    torch.testing.assert_close(res.cpu().float(), rr.float(), atol=0, rtol=0)
    torch.testing.assert_close(x.cpu().float(), xr.float(), atol=2e-2, rtol=1.6e-2)


@pytest.mark.parametrize("T,I", [(1, 1024), (64, 14336), (5, 3584), (3, 8)])
def test_silu_and_mul(T, I):
    torch.manual_seed(2)
    x = torch.randn(T, 2 * I, device="cuda", dtype=torch.bfloat16) * 2
    y = ops.silu_and_mul(x)
    torch.testing.assert_close(y.cpu().float(), ref.silu_and_mul(x.cpu()).float(), atol=2e-2, rtol=1.6e-2)


def test_native_library_is_loaded():
    from polykey_service_amd.ops import native
    assert native.lib().pk_kernels_abi_version() == 1
    with open("/proc/self/maps") as f:
        assert "libpk_kernels.so" in f.read()


@pytest.mark.parametrize("start,local", [(0, 1000), (250, 300)])
def test_embedding_vocab_parallel_mask(start, local):
    from polykey_service_amd import ops
    V, H, T = 1000, 4096, 77
    table = torch.randn(local, H, device="cuda").to(torch.bfloat16)
    ids = torch.randint(0, V, (T,), device="cuda", dtype=torch.int32)
    y = ops.embedding(ids, table, start, local)
    loc = ids.long() - start
    mask = (loc >= 0) & (loc < local)
    exp = torch.where(mask[:, None], table[loc.clamp(0, local - 1)], torch.zeros_like(table[:1]))
    assert torch.equal(y, exp)
