"""Prometheus metrics (``prometheus_client``) on a side port.

The reference only recommends Prometheus (``test/README.md:61-70``); here the server exports
RPC latency/count by method and code (fed by the logging interceptor's observer), and the
engine exports request TTFT / inter-token latency / end-to-end latency histograms, output
token and request counters, queue depth, running batch size and KV-block utilisation
(SURVEY.md §5.5).
"""
from __future__ import annotations

from typing import Optional

from prometheus_client import CollectorRegistry, Counter, Gauge, Histogram, start_http_server

_LAT_BUCKETS = (.001, .0025, .005, .01, .025, .05, .1, .25, .5, 1, 2.5, 5, 10, 30, 60, 120)
_TOK_BUCKETS = (.002, .004, .006, .008, .01, .015, .02, .03, .05, .1, .25, .5, 1)

_current: Optional["Metrics"] = None


class Metrics:
    def __init__(self, registry: Optional[CollectorRegistry] = None):
        self.registry = registry or CollectorRegistry()
        r = self.registry
        self.rpc_latency = Histogram("polykey_rpc_latency_seconds", "gRPC call latency", ["method", "code"],
                                     buckets=_LAT_BUCKETS, registry=r)
        self.requests = Counter("polykey_llm_requests_total", "finished LLM requests", ["finish_reason"], registry=r)
        self.output_tokens = Counter("polykey_llm_output_tokens_total", "generated tokens", registry=r)
        self.ttft = Histogram("polykey_llm_ttft_seconds", "time to first token", buckets=_LAT_BUCKETS, registry=r)
        self.itl = Histogram("polykey_llm_inter_token_seconds", "mean inter-token latency per request",
                             buckets=_TOK_BUCKETS, registry=r)
        self.e2e = Histogram("polykey_llm_e2e_seconds", "request end-to-end latency", buckets=_LAT_BUCKETS,
                             registry=r)
        self.running = Gauge("polykey_engine_running_seqs", "sequences in the running batch", registry=r)
        self.waiting = Gauge("polykey_engine_waiting_seqs", "queued sequences", registry=r)
        self.kv_util = Gauge("polykey_engine_kv_utilization", "fraction of KV blocks in use", registry=r)
        self.step_seconds = Histogram("polykey_engine_step_seconds", "engine step wall time", buckets=_TOK_BUCKETS,
                                      registry=r)
        # cumulative engine counts exported as Counters (advanced by the delta since the last step)
        self.preemptions = Counter("polykey_engine_preemptions", "sequences preempted (KV recompute)", registry=r)
        self.cached_tokens = Counter("polykey_engine_prefix_cache_hit_tokens", "prompt tokens served from the "
                                     "prefix cache", registry=r)
        self.prefix_queries = Counter("polykey_engine_prefix_cache_queries", "full prompt blocks looked up in the "
                                      "prefix cache", registry=r)
        self.prefix_hits = Counter("polykey_engine_prefix_cache_hits", "prompt blocks served from the prefix cache",
                                   registry=r)
        self.prefix_collisions = Counter("polykey_engine_prefix_cache_rejected", "hash matches rejected by the "
                                         "token / parent check", registry=r)
        self._last: dict = {}
        self.cached_blocks = Gauge("polykey_engine_prefix_cache_blocks", "KV blocks registered in the prefix cache",
                                   registry=r)

    def _advance(self, counter, key: str, total: int) -> None:
        """Counter += growth of an engine-side cumulative count (a restarted engine's count
        starting over from 0 is taken as growth from 0)."""
        prev = self._last.get(key, 0)
        delta = total - prev if total >= prev else total
        if delta > 0:
            counter.inc(delta)
        self._last[key] = total

    @classmethod
    def start(cls, addr: str) -> "Metrics":
        m = cls()
        host, _, port = addr.rpartition(":")
        start_http_server(int(port), addr=host or "0.0.0.0", registry=m.registry)
        set_current(m)
        return m

    def observe_rpc(self, method: str, seconds: float, code: str) -> None:
        self.rpc_latency.labels(method, code).observe(seconds)

    def observe_step(self, engine, seconds: float, outputs) -> None:
        sch = engine.scheduler
        self.step_seconds.observe(seconds)
        self.running.set(len(sch.running))
        self.waiting.set(len(sch.waiting))
        bm = engine.bm
        self.kv_util.set(1.0 - bm.num_free / max(bm.num_blocks, 1))
        self._advance(self.preemptions, "preemptions", sch.num_preemptions)
        self._advance(self.cached_tokens, "tokens", getattr(sch, "num_cached_tokens", 0))
        self._advance(self.prefix_queries, "queries", getattr(bm, "prefix_queries", 0))
        self._advance(self.prefix_hits, "hits", getattr(bm, "prefix_hits", 0))
        self._advance(self.prefix_collisions, "collisions", getattr(bm, "prefix_collisions", 0))
        self.cached_blocks.set(getattr(bm, "num_cached", 0))
        n = 0
        for o in outputs:
            n += len(o.new_token_ids)
            if o.finished:
                self.requests.labels(o.finish_reason or "unknown").inc()
                m = o.metrics or {}
                if m.get("ttft_s") is not None:
                    self.ttft.observe(m["ttft_s"])
                if m.get("mean_itl_s") is not None:
                    self.itl.observe(m["mean_itl_s"])
                if m.get("e2e_s") is not None:
                    self.e2e.observe(m["e2e_s"])
        self.output_tokens.inc(n)


def current() -> Optional[Metrics]:
    return _current


def set_current(m: Optional[Metrics]) -> None:
    global _current
    _current = m
