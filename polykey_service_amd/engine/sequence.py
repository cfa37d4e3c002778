"""Request / sequence state for the continuous-batching engine."""
from __future__ import annotations

import dataclasses
import enum
import itertools
import time
from typing import List, Optional, Sequence as Seq


@dataclasses.dataclass
class SamplingParams:
    max_tokens: int = 16
    temperature: float = 0.0      # 0 → greedy
    top_p: float = 1.0
    top_k: int = 0
    min_p: float = 0.0
    seed: Optional[int] = None
    stop_token_ids: Seq[int] = ()
    ignore_eos: bool = False
    stop: Seq[str] = ()           # stop strings (checked on detokenized text)
    cache_salt: Optional[str] = None  # prefix-cache namespace (e.g. a tenant id); None = shared

    def validate(self, max_model_len: int) -> None:
        if self.max_tokens < 1:
            raise ValueError("max_tokens must be >= 1")
        if self.temperature < 0:
            raise ValueError("temperature must be >= 0")
        if not 0 < self.top_p <= 1:
            raise ValueError("top_p must be in (0, 1]")
        if self.top_k < 0:
            raise ValueError("top_k must be >= 0")
        if not 0 <= self.min_p < 1:
            raise ValueError("min_p must be in [0, 1)")

    @classmethod
    def from_dict(cls, d: dict) -> "SamplingParams":
        kw = {}
        for f in dataclasses.fields(cls):
            if f.name in d and d[f.name] is not None:
                v = d[f.name]
                if f.name in ("max_tokens", "top_k"):
                    v = int(v)
                elif f.name in ("temperature", "top_p", "min_p"):
                    v = float(v)
                elif f.name == "seed":
                    v = int(v)
                elif f.name in ("stop_token_ids",):
                    v = tuple(int(x) for x in v)
                elif f.name == "stop":
                    v = (v,) if isinstance(v, str) else tuple(v)
                elif f.name == "ignore_eos":
                    v = bool(v)
                elif f.name == "cache_salt":
                    v = str(v)
                kw[f.name] = v
        return cls(**kw)


class SeqStatus(enum.Enum):
    WAITING = 0
    RUNNING = 1
    FINISHED = 2


class FinishReason(str, enum.Enum):
    LENGTH = "length"
    STOP = "stop"
    ABORT = "abort"
    ERROR = "error"


_ids = itertools.count(1)


class Sequence:
    __slots__ = ("seq_id", "request_id", "prompt_ids", "output_ids", "params", "status", "num_computed",
                 "arrival", "first_scheduled", "first_token_time", "finish_time", "finish_reason",
                 "num_preemptions", "eos_token_id", "token_times", "user", "num_cached_tokens",
                 "cache_salt")

    def __init__(self, request_id: str, prompt_ids: List[int], params: SamplingParams, eos_token_id: int = -1,
                 user=None, cache_salt: Optional[str] = None):
        self.seq_id = next(_ids)
        self.request_id = request_id
        self.prompt_ids = list(prompt_ids)
        self.output_ids: List[int] = []
        self.params = params
        self.status = SeqStatus.WAITING
        self.num_computed = 0
        self.arrival = time.monotonic()
        self.first_scheduled: Optional[float] = None
        self.first_token_time: Optional[float] = None
        self.finish_time: Optional[float] = None
        self.finish_reason: Optional[FinishReason] = None
        self.num_preemptions = 0
        self.num_cached_tokens = 0  # tokens whose KV came from the prefix cache
        self.eos_token_id = eos_token_id
        self.token_times: List[float] = []
        self.user = user
        # prefix-cache namespace (Scheduler._salt); None = the request's params.cache_salt
        self.cache_salt = cache_salt if cache_salt is not None else getattr(params, "cache_salt", None)

    @property
    def num_tokens(self) -> int:
        return len(self.prompt_ids) + len(self.output_ids)

    @property
    def num_pending(self) -> int:
        """Tokens whose KV is not yet in the cache."""
        return self.num_tokens - self.num_computed

    def token_slice(self, start: int, end: int) -> List[int]:
        n = len(self.prompt_ids)
        if end <= n:
            return self.prompt_ids[start:end]
        if start >= n:
            return self.output_ids[start - n:end - n]
        return self.prompt_ids[start:] + self.output_ids[:end - n]

    @property
    def seed(self) -> int:
        return (self.params.seed if self.params.seed is not None else self.seq_id * 2654435761) & 0x7FFFFFFF

    def is_finished(self) -> bool:
        return self.status == SeqStatus.FINISHED

    def append_token(self, tok: int, now: float) -> Optional[FinishReason]:
        self.output_ids.append(tok)
        self.token_times.append(now)
        if self.first_token_time is None:
            self.first_token_time = now
        p = self.params
        if not p.ignore_eos and (tok == self.eos_token_id or tok in p.stop_token_ids):
            return FinishReason.STOP
        if len(self.output_ids) >= p.max_tokens:
            return FinishReason.LENGTH
        return None


@dataclasses.dataclass
class RequestOutput:
    request_id: str
    new_token_ids: List[int]
    finished: bool
    finish_reason: Optional[str] = None
    num_prompt_tokens: int = 0
    num_output_tokens: int = 0
    metrics: Optional[dict] = None


def seq_metrics(s: Sequence) -> dict:
    t0 = s.arrival
    ttft = (s.first_token_time - t0) if s.first_token_time else None
    e2e = (s.finish_time - t0) if s.finish_time else None
    itl = None
    if len(s.token_times) > 1:
        itl = (s.token_times[-1] - s.token_times[0]) / (len(s.token_times) - 1)
    return {
        "queue_s": (s.first_scheduled - t0) if s.first_scheduled else None,
        "ttft_s": ttft, "e2e_s": e2e, "mean_itl_s": itl, "preemptions": s.num_preemptions,
        "cached_prompt_tokens": s.num_cached_tokens,
    }
