"""Hot ops: hand-written gfx950 HIP kernels (``csrc/kernels``) with fp32 references."""
from . import reference
from .embedding import embedding
from .norm import fused_add_rms_norm, rms_norm, silu_and_mul

__all__ = ["reference", "embedding", "fused_add_rms_norm", "rms_norm", "silu_and_mul"]
