"""Model families: Llama-3 (8B / 70B) and Mixtral-8x7B, TP/EP-aware."""
from .config import PRESETS, ModelConfig, get_config
from .llama import LlamaForCausalLM


def build_model(cfg: ModelConfig, st, dtype, device):
    if cfg.is_moe:
        from .mixtral import MixtralForCausalLM
        return MixtralForCausalLM(cfg, st, dtype, device)
    return LlamaForCausalLM(cfg, st, dtype, device)


__all__ = ["PRESETS", "ModelConfig", "get_config", "LlamaForCausalLM", "build_model"]
