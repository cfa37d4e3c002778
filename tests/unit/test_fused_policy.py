"""Which decode launches a rank may fuse: a fused launch that loses its
in-launch hand-off falls back to the two-launch path only at TP = 1 (llm_engine.py
_complete_or_redo), so a TP rank that shares its GPU with co-tenants -- the only place a hand-off
can be starved -- must not take the fused QKV -> attention launch (nor the fused MLP)."""
import torch

from polykey_service_amd.models import build_model, get_config
from polykey_service_amd.ops import attention as A
from polykey_service_amd.ops import gemm
from polykey_service_amd.parallel.state import ParallelState


def _md(T):
    return A.AttnMetadata(num_decode=T, num_prefill=0, num_prefill_tokens=0, max_prefill_q_len=0,
                          slot_mapping=None)


def test_tp_rank_on_a_shared_gpu_keeps_two_launches(monkeypatch):
    monkeypatch.setattr(gemm, "QKV_ATTN_MIN_KV", 1)
    cfg = get_config("tiny-llama-gqa4")
    for tp, shared, ok in ((1, False, True), (1, True, True), (2, False, True), (2, True, False)):
        st = ParallelState(tp_size=tp, tp_rank=0, device=torch.device("cpu"))
        st.shared_device = shared
        m = build_model(cfg, st, torch.bfloat16, torch.device("cpu"))
        at = m.layers[0].attn
        assert m._qkv_attn_fused_ok(at, 8, cfg.hidden_size // gemm.PART_COLS, _md(8)) is ok, (tp, shared)
