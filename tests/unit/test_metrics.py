"""Prometheus metrics wiring (RPC observer + engine step observer)."""
from prometheus_client import generate_latest

from polykey_service_amd.engine.sequence import RequestOutput
from polykey_service_amd.utils.metrics import Metrics


class _BM:
    num_free, num_blocks, num_cached = 30, 40, 5
    prefix_queries, prefix_hits, prefix_collisions = 12, 7, 1


class _Sch:
    running, waiting, num_preemptions, num_cached_tokens = [1, 2], [3], 2, 160


class _Eng:
    bm, scheduler = _BM(), _Sch()


def test_metrics_export():
    m = Metrics()
    m.observe_rpc("/polykey.v2.PolykeyService/ExecuteTool", 0.01, "OK")
    outs = [RequestOutput("a", [5], False), RequestOutput("b", [6], True, "length", 3, 4,
                                                          {"ttft_s": 0.1, "mean_itl_s": 0.01, "e2e_s": 0.2})]
    m.observe_step(_Eng(), 0.005, outs)
    text = generate_latest(m.registry).decode()
    assert 'polykey_rpc_latency_seconds_count{code="OK",method="/polykey.v2.PolykeyService/ExecuteTool"} 1.0' in text
    assert "polykey_llm_output_tokens_total 2.0" in text
    assert 'polykey_llm_requests_total{finish_reason="length"} 1.0' in text
    assert "polykey_engine_kv_utilization 0.25" in text
    assert "polykey_engine_running_seqs 2.0" in text and "polykey_llm_ttft_seconds_count 1.0" in text
    assert "polykey_engine_prefix_cache_hit_tokens_total 160.0" in text
    assert "polykey_engine_prefix_cache_blocks 5.0" in text
    assert "polykey_engine_prefix_cache_queries_total 12.0" in text and "polykey_engine_prefix_cache_hits_total 7.0" in text
    # counters advance by the growth of the engine's cumulative counts
    eng = _Eng()
    eng.scheduler.num_cached_tokens = 200
    m.observe_step(eng, 0.005, [])
    eng.scheduler.num_cached_tokens = 160  # counts do not go down: the counter holds
    text = generate_latest(m.registry).decode()
    assert "polykey_engine_prefix_cache_hit_tokens_total 200.0" in text
