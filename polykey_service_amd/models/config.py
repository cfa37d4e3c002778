"""Model architecture presets (public HF configs; SURVEY.md §2.3 "Model constants").

The reference has no models; these are the north-star families (``BASELINE.json:8-11``):
Llama-3-8B, Llama-3-70B and Mixtral-8x7B, plus tiny variants with the same structure used by
tests (head_dim stays 128 because the attention kernels are specialised for it).
"""
from __future__ import annotations

import dataclasses
import json
import os
from typing import Dict, Optional


@dataclasses.dataclass(frozen=True)
class ModelConfig:
    name: str
    vocab_size: int
    hidden_size: int
    intermediate_size: int
    num_layers: int
    num_heads: int
    num_kv_heads: int
    head_dim: int = 128
    rope_theta: float = 500000.0
    rms_eps: float = 1e-5
    max_position: int = 8192
    num_experts: int = 0          # 0 → dense MLP
    experts_per_token: int = 2
    tie_embeddings: bool = False
    rope_scaling: Optional[dict] = None
    bos_token_id: int = 128000
    eos_token_id: int = 128001
    init_std: float = 0.02
    # random-init std of the MoE router (None: init_std).  The tiny test MoEs use a wide router so
    # top-2 routing has no near-ties that bf16 reduction-order noise could flip between TP layouts
    router_init_std: Optional[float] = None

    @property
    def is_moe(self) -> bool:
        return self.num_experts > 0

    @property
    def q_size(self) -> int:
        return self.num_heads * self.head_dim

    @property
    def kv_size(self) -> int:
        return self.num_kv_heads * self.head_dim

    def num_params(self) -> int:
        H, I, L, V = self.hidden_size, self.intermediate_size, self.num_layers, self.vocab_size
        attn = H * (self.q_size + 2 * self.kv_size) + self.q_size * H
        mlp = 3 * H * I * (self.num_experts or 1) + (H * self.num_experts if self.is_moe else 0)
        emb = V * H * (1 if self.tie_embeddings else 2)
        return L * (attn + mlp + 2 * H) + emb + H

    def kv_bytes_per_token(self, dtype_bytes: int = 2) -> int:
        return 2 * self.num_layers * self.kv_size * dtype_bytes


PRESETS: Dict[str, ModelConfig] = {
    "llama3-8b": ModelConfig("llama3-8b", 128256, 4096, 14336, 32, 32, 8),
    "llama3-70b": ModelConfig("llama3-70b", 128256, 8192, 28672, 80, 64, 8),
    "mixtral-8x7b": ModelConfig("mixtral-8x7b", 32000, 4096, 14336, 32, 32, 8, rope_theta=1e6,
                                max_position=32768, num_experts=8, experts_per_token=2,
                                bos_token_id=1, eos_token_id=2),
    # test-sized models with the real structure (GQA groups 4 and 8, MoE top-2)
    "tiny-llama": ModelConfig("tiny-llama", 1024, 512, 1024, 2, 4, 1, max_position=2048, init_std=0.05,
                              bos_token_id=1, eos_token_id=2),
    "tiny-llama-gqa4": ModelConfig("tiny-llama-gqa4", 1024, 1024, 2048, 2, 8, 2, max_position=2048,
                                   init_std=0.05, bos_token_id=1, eos_token_id=2),
    "tiny-mixtral": ModelConfig("tiny-mixtral", 1024, 512, 768, 2, 8, 2, rope_theta=1e6, max_position=2048,
                                num_experts=4, experts_per_token=2, init_std=0.05, bos_token_id=1,
                                eos_token_id=2, router_init_std=0.5),
    # the 70B TP=8 per-rank shape at test size: 8 KV heads (one per rank at TP=8), GQA group 8,
    # vocab not divisible by 8 (padded shards, like 128256 / 8 = 16032 rows), hidden % 1024 == 0
    "tiny-llama-g8": ModelConfig("tiny-llama-g8", 1003, 1024, 2048, 2, 64, 8, max_position=2048, init_std=0.05,
                                 bos_token_id=1, eos_token_id=2),
    # Mixtral's expert count and attention shape (8 experts: one per rank at EP=8, 8 KV heads)
    "tiny-mixtral-e8": ModelConfig("tiny-mixtral-e8", 1000, 1024, 1024, 2, 32, 8, rope_theta=1e6,
                                   max_position=2048, num_experts=8, experts_per_token=2, init_std=0.05,
                                   bos_token_id=1, eos_token_id=2, router_init_std=0.5),
    "small-llama": ModelConfig("small-llama", 32000, 2048, 5632, 8, 16, 4, init_std=0.02,
                               bos_token_id=1, eos_token_id=2),
}


def get_config(name_or_path: str) -> ModelConfig:
    if name_or_path in PRESETS:
        return PRESETS[name_or_path]
    path = os.path.join(name_or_path, "config.json") if os.path.isdir(name_or_path) else name_or_path
    if os.path.isfile(path):
        return from_hf_config(path)
    raise KeyError(f"unknown model {name_or_path!r}; presets: {sorted(PRESETS)}")


def from_hf_config(path: str) -> ModelConfig:
    with open(path) as f:
        c = json.load(f)
    nh = c["num_attention_heads"]
    eos = c.get("eos_token_id", 2)
    return ModelConfig(
        name=c.get("_name_or_path", os.path.basename(os.path.dirname(path)) or "hf-model"),
        vocab_size=c["vocab_size"], hidden_size=c["hidden_size"], intermediate_size=c["intermediate_size"],
        num_layers=c["num_hidden_layers"], num_heads=nh, num_kv_heads=c.get("num_key_value_heads", nh),
        head_dim=c.get("head_dim", c["hidden_size"] // nh), rope_theta=c.get("rope_theta", 10000.0),
        rms_eps=c.get("rms_norm_eps", 1e-5), max_position=c.get("max_position_embeddings", 8192),
        num_experts=c.get("num_local_experts", 0), experts_per_token=c.get("num_experts_per_tok", 2),
        tie_embeddings=c.get("tie_word_embeddings", False), rope_scaling=c.get("rope_scaling"),
        bos_token_id=c.get("bos_token_id", 1) or 1, eos_token_id=eos[0] if isinstance(eos, list) else eos)
