"""Checkpoint round trip: random-init model → HF-format safetensors → load_hf (TP=1 and TP-sliced)."""
import pytest
import torch

from polykey_service_amd.engine import EngineConfig, LLMEngine, SamplingParams
from polykey_service_amd.models import build_model, get_config
from polykey_service_amd.parallel.state import ParallelState


@pytest.mark.parametrize("name", ["tiny-llama-gqa4", "tiny-mixtral"])
def test_save_load_roundtrip(tmp_path, name):
    cfg = get_config(name)
    st = ParallelState()
    a = build_model(cfg, st, torch.bfloat16, torch.device("cpu")).init_random(11)
    a.save_hf(str(tmp_path))
    cfg2 = get_config(str(tmp_path))
    assert cfg2.num_experts == cfg.num_experts and cfg2.num_kv_heads == cfg.num_kv_heads
    b = build_model(cfg2, st, torch.bfloat16, torch.device("cpu")).load_hf(str(tmp_path))
    sa, sb = dict(a.named_parameters()), dict(b.named_parameters())
    assert sa.keys() == sb.keys()
    for k in sa:
        assert torch.equal(sa[k], sb[k]), k


def test_engine_from_checkpoint_dir(tmp_path):
    cfg = get_config("tiny-llama")
    a = build_model(cfg, ParallelState(), torch.bfloat16, torch.device("cpu")).init_random(5)
    a.save_hf(str(tmp_path))
    kw = dict(max_num_seqs=4, max_num_batched_tokens=64, max_model_len=256, hip_graphs=False, device="cpu")
    e1 = LLMEngine(EngineConfig(model="tiny-llama", seed=5, **kw), ParallelState())
    e2 = LLMEngine(EngineConfig(model="tiny-llama", model_path=str(tmp_path), **kw), ParallelState())
    p = [[1, 7, 8, 9]]
    assert e1.generate(p, SamplingParams(max_tokens=5)) == e2.generate(p, SamplingParams(max_tokens=5))
