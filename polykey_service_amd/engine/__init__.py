from .llm_engine import EngineConfig, LLMEngine
from .sequence import FinishReason, RequestOutput, SamplingParams, Sequence

__all__ = ["EngineConfig", "LLMEngine", "FinishReason", "RequestOutput", "SamplingParams", "Sequence"]
