"""CPU reference ops: paged K-cache layout."""
import pytest



def test_kcache_fragment_layout():
    """The paged K cache keeps each 32-token tile in MFMA fragment order: lane l of load (t, kk)
    of the attention kernels reads 8 dims of key 8*((l&15)>>2) + 4t + (l&3) -- a bijection
    within every tile of a block (common.h kcache_off)."""
    from polykey_service_amd.ops.reference import k_cache_logical, kcache_index
    for bs in (32, 64, 96):
        idx = kcache_index(bs)
        assert sorted(idx.view(-1).tolist()) == list(range(bs * 128))
    idx = kcache_index(32)
    for t in range(2):
        for kk in range(4):
            for lane in range(64):
                r, g = lane & 15, lane >> 4
                tok = 8 * (r >> 2) + 4 * t + (r & 3)
                for j in range(8):
                    assert idx[tok, 32 * g + 8 * kk + j] == ((t * 4 + kk) * 64 + lane) * 8 + j
    # rope_and_cache writes through the layout; k_cache_logical reads it back
    import torch
    from polykey_service_amd.ops import reference as R
    nq, nkv, T, bs = 2, 2, 5, 64
    qkv = torch.randn(T, (nq + 2 * nkv) * 128)
    kc = torch.zeros(3, nkv, bs, 128)
    vc = torch.zeros(3, nkv, 128, bs)
    slots = torch.tensor([0, 63, 64, 100, 191], dtype=torch.int32)
    pos = torch.arange(T, dtype=torch.int32)
    cs = R.rope_cos_sin_cache(64, 128, 10000.0, None)
    q = qkv.clone()
    R.rope_and_cache(q, pos, cs, kc, vc, slots, nq, nkv, 128)
    k = q.view(T, nq + 2 * nkv, 128)[:, nq:nq + nkv]
    logical = k_cache_logical(kc)
    for i, s in enumerate(slots.tolist()):
        assert torch.equal(logical[s // bs, :, s % bs], k[i])
    with pytest.raises(ValueError):
        kcache_index(16)


def test_vcache_fragment_layout():
    """The paged V cache keeps each 32-token tile as [d / 16][key / 8][d % 16][key % 8]: lane
    (r, g) of d-tile dt reads keys 8g..8g+7 of channel 16 dt + r as 16 contiguous bytes, the
    wave's 64 lanes one contiguous KiB (common.h vcache_off); a bijection within every tile."""
    import torch
    from polykey_service_amd.ops import reference as R
    for bs in (32, 64, 96):
        idx = R.vcache_index(bs)
        assert sorted(idx.view(-1).tolist()) == list(range(bs * 128))
    idx = R.vcache_index(32)
    for dt in range(8):
        for lane in range(64):
            r, g = lane & 15, lane >> 4
            for j in range(8):
                assert idx[8 * g + j, 16 * dt + r] == dt * 512 + lane * 8 + j
    nq, nkv, T, bs = 2, 2, 5, 64
    qkv = torch.randn(T, (nq + 2 * nkv) * 128)
    kc = torch.zeros(3, nkv, bs, 128)
    vc = torch.zeros(3, nkv, 128, bs)
    slots = torch.tensor([0, 63, 64, 100, 191], dtype=torch.int32)
    R.rope_and_cache(qkv.clone(), torch.arange(T, dtype=torch.int32), R.rope_cos_sin_cache(64, 128, 10000.0, None),
                     kc, vc, slots, nq, nkv, 128)
    v = qkv.view(T, nq + 2 * nkv, 128)[:, nq + nkv:]
    logical = R.v_cache_logical(vc)
    for i, s in enumerate(slots.tolist()):
        assert torch.equal(logical[s // bs, :, s % bs], v[i])
    with pytest.raises(ValueError):
        R.vcache_index(16)
