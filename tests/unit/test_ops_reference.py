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
