"""Block-packed decode-GEMM weight layout (ops/gemm.py pack_weight) — pure tensor logic, CPU.

The kernel (csrc/kernels/gemm_skinny.hip, PK path) reads, for n-block nb, k-step ks (128
deep), row tile t of the block and k-block s (32 deep), the 1 KiB fragment at element offset
``nb*128*K + (ks*32 + t*4 + s)*512`` where lane l = 16*g + r holds W[nb*128 + 16t + r][ks*128 +
32s + 8g .. +8].  These tests pin that contract."""
import torch

from polykey_service_amd.ops import gemm


def test_roundtrip():
    w = torch.randn(384, 768)
    assert torch.equal(gemm.unpack_weight(gemm.pack_weight(w)), w)


def test_fragment_addressing_matches_kernel():
    N, K = 256, 512
    w = torch.arange(N * K, dtype=torch.float32).view(N, K)
    flat = gemm.pack_weight(w).view(-1)
    for nb, ks, t, s in ((0, 0, 0, 0), (1, 2, 3, 1), (1, 3, 7, 3), (0, 1, 5, 2)):
        off = nb * 128 * K + (ks * 32 + t * 4 + s) * 512
        frag = flat[off:off + 512].view(64, 8)
        for lane in (0, 5, 16, 17, 40, 63):
            g, r = lane // 16, lane % 16
            row = nb * 128 + 16 * t + r
            k0 = ks * 128 + 32 * s + 8 * g
            assert torch.equal(frag[lane], w[row, k0:k0 + 8]), (nb, ks, t, s, lane)


def test_workgroup_stream_is_contiguous():
    """A workgroup's bytes for one k-step (8 tiles x 4 k-blocks) form one 32 KiB run."""
    N, K = 256, 256
    w = torch.arange(N * K, dtype=torch.float32).view(N, K)
    flat = gemm.pack_weight(w).view(-1)
    nb, ks = 1, 1
    run = flat[nb * 128 * K + ks * 32 * 512:][:32 * 512].view(8, 4, 64, 8)
    rows = {int(v) // K for v in run.flatten()}
    cols = {int(v) % K for v in run.flatten()}
    assert rows == set(range(128, 256)) and cols == set(range(128, 256))


def test_nt_bit_threshold(monkeypatch):
    monkeypatch.setattr(gemm, "NT_MIN_BYTES", 1 << 20)
    small = torch.empty(128, 128, dtype=torch.bfloat16)
    big = torch.empty(1024, 1024, dtype=torch.bfloat16)
    assert gemm._wmode(None) == 0
    assert gemm._wmode(small) == gemm.PACKED_BIT
    assert gemm._wmode(big) == gemm.PACKED_BIT | gemm.NT_BIT
