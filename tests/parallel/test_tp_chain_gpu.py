"""The TP decode chain at the 70B TP=8 per-rank shapes (H 8192, 8 q / 1 kv heads, gate_up 7168 x
8192 split over K, down 8192 x 3584), one rank on one GPU with the collectives reduced to their
local half (tools/tp_solo.py SoloAR): the fused launches (QKV -> attention, gate_up -> down) give
hidden states and KV caches bit-identical to the two-launch chain, and the step really ran them.
(Serving keeps them off at this shape -- measured slower, profiles/r4_tp_solo.md -- the test
turns them on.)"""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _run(model, md, kv, ids, pos):
    with torch.inference_mode():
        h = model(ids, pos, md, kv)
        torch.cuda.synchronize()
    return h.clone()


def test_tp8_shard_fused_chain_bit_identical_to_two_launches(monkeypatch):
    import dataclasses

    from polykey_service_amd.models import build_model, get_config
    from polykey_service_amd.ops import attention as A
    from polykey_service_amd.ops import gemm
    from polykey_service_amd.parallel.state import ParallelState, get_state, set_state
    from tools.tp_solo import SoloAR

    old = get_state()
    dev = torch.device("cuda:0")
    st = ParallelState(tp_size=8, tp_rank=0, device=dev)
    st.custom_ar = SoloAR(8)
    set_state(st)
    saved = (gemm.MLP_FUSED, gemm.QKV_ATTN_FUSED)
    try:
        cfg = dataclasses.replace(get_config("llama3-70b"), num_layers=2)
        model = build_model(cfg, st, torch.bfloat16, dev).init_random(5)
        with torch.no_grad():  # non-uniform norms: the folds are not no-ops
            for layer in model.layers:
                layer.ln1.mul_(torch.linspace(0.6, 1.4, layer.ln1.numel(), device=dev).to(layer.ln1.dtype))
                layer.ln2.mul_(torch.linspace(1.4, 0.6, layer.ln2.numel(), device=dev).to(layer.ln2.dtype))
        model.pack_decode_weights()
        at = model.layers[0].attn
        assert (at.nq, at.nkv) == (8, 1)
        B, BS, ctx = 64, 32, 200
        maxb = (ctx + BS) // BS + 1
        bt = torch.arange(B * maxb, dtype=torch.int32, device=dev).view(B, maxb)
        cl = torch.arange(ctx - B, ctx, dtype=torch.int32, device=dev) + 1
        pos = cl - 1
        slots = torch.stack([bt[i, int(p) // BS] * BS + int(p) % BS for i, p in enumerate(pos.tolist())]).int()
        po, pml = A.decode_workspace(B, at.nq, maxb, BS, dev)
        md = A.AttnMetadata(num_decode=B, num_prefill=0, num_prefill_tokens=0, max_prefill_q_len=0,
                            slot_mapping=slots, decode_block_tables=bt, decode_context_lens=cl, decode_part_o=po,
                            decode_part_ml=pml)
        gen = torch.Generator(device=dev).manual_seed(1)
        kv0 = [((torch.randn(B * maxb, 1, BS, 128, device=dev, generator=gen) * 0.5).to(torch.bfloat16),
                (torch.randn(B * maxb, 1, 128, BS, device=dev, generator=gen) * 0.5).to(torch.bfloat16))
               for _ in model.layers]
        ids = torch.randint(0, cfg.vocab_size, (B,), dtype=torch.int32, device=dev)
        calls = {"mlp": 0, "qkv": 0}
        real_mlp, real_qkv = gemm.mlp_fused, gemm.qkv_attn_fused

        def mlp(*a, **k):
            calls["mlp"] += 1
            return real_mlp(*a, **k)

        def qkv(*a, **k):
            calls["qkv"] += 1
            return real_qkv(*a, **k)
        monkeypatch.setattr(gemm, "mlp_fused", mlp)
        monkeypatch.setattr(gemm, "qkv_attn_fused", qkv)
        # the serving policy keeps the QKV -> attention launch off at this shape (one kv head per
        # rank: measured slower, gemm.QKV_ATTN_MIN_KV); it must still be exact where allowed.  The
        # fused MLP never takes the shard's K-split gate_up (that variant was removed in round 6)
        monkeypatch.setattr(gemm, "QKV_ATTN_MIN_KV", 1)
        # the fused launch's QKV tiles are 128-row n-blocks at the full split: compare with the same
        # tiling (the two-launch chain's half-split QKV sums its slabs in another grouping)
        monkeypatch.setattr(gemm, "QKV_HALF", False)
        outs = []
        for fused in (False, True):
            gemm.MLP_FUSED = gemm.QKV_ATTN_FUSED = fused
            kv = [(k.clone(), v.clone()) for k, v in kv0]
            outs.append((_run(model, md, kv, ids, pos), kv))
        assert calls == {"mlp": 0, "qkv": 2}, calls  # both layers took the fused QKV -> attention launch
        (h0, kv_a), (h1, kv_b) = outs
        assert torch.equal(h0, h1)
        for (ka, va), (kb, vb) in zip(kv_a, kv_b):
            assert torch.equal(ka, kb) and torch.equal(va, vb)
        assert torch.isfinite(h1.float()).all() and h1.float().abs().max() > 0
        gemm.check_fused()
    finally:
        gemm.MLP_FUSED, gemm.QKV_ATTN_FUSED = saved
        set_state(old)
