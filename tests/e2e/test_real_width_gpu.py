"""Correctness at the REAL Llama-3-8B widths: a 2-layer model with hidden
4096, 32 q / 8 kv heads, intermediate 14336 and the full 128,256-token vocabulary, run by the GPU
engine -- prefill on hipBLASLt + the hand-written attention / norm / RoPE kernels, decode on the
fully fused chain (RMSNorm weights folded into block-packed QKV / gate-up, QKV split-K slabs
consumed by the decode attention kernel with RoPE and the cache write folded in, o-projection
slabs from 64-row n-blocks, residual-update kernels, packed LM head) -- against the fp32 CPU
reference engine on the same weights.  The norm weights are made non-uniform so folding them
is not a no-op."""
import copy
import dataclasses

import pytest
import torch

from polykey_service_amd.engine import EngineConfig, LLMEngine, SamplingParams
from polykey_service_amd.models import build_model, get_config
from polykey_service_amd.parallel.state import ParallelState

pytestmark = pytest.mark.gpu

PROMPTS = [[128000] + list(range(1000, 1000 + n)) for n in (5, 37, 70)]
# the headline decode shape: 64 sequences (the fused launches' 4 x 16-row tile), and 40 (3 tiles)
MANY = {n: [[128000] + [(97 * i + 13 * j) % 20000 + 500 for j in range(3 + i % 13)] for i in range(n)] for n in (40, 64)}


def _engine(model, dev, cfg, n=8):
    e = LLMEngine(EngineConfig(model="llama3-8b", num_layers=cfg.num_layers, max_num_seqs=max(8, n),
                               max_num_batched_tokens=2048, max_model_len=1024, num_kv_blocks=256, hip_graphs=False,
                               device=dev, prefix_caching=False), ParallelState(device=torch.device(dev)), model=model)
    e.runner.keep_logits = True
    return e


def _two_steps(e, prompts=PROMPTS):
    for p in prompts:
        e.add_request(p, SamplingParams(max_tokens=2, ignore_eos=True))
    e.step()
    prefill = e.runner.last_logits.float().cpu().clone()
    seqs = list(e.scheduler.running)
    first = [s.output_ids[0] for s in sorted(seqs, key=lambda s: s.seq_id)]
    e.step()
    decode = e.runner.last_logits.float().cpu().clone()
    return prefill, first, decode


@pytest.mark.parametrize("n", [3, 40, 64])
def test_llama3_8b_width_prefill_and_fused_decode_match_cpu_reference(n):
    prompts = PROMPTS if n == 3 else MANY[n]
    cfg = dataclasses.replace(get_config("llama3-8b"), num_layers=2)
    cpu = build_model(cfg, ParallelState(), torch.bfloat16, torch.device("cpu")).init_random(11)
    with torch.no_grad():
        for layer in cpu.layers:
            layer.ln1.copy_(torch.linspace(0.5, 1.5, layer.ln1.numel()).to(layer.ln1.dtype))
            layer.ln2.copy_(torch.linspace(1.5, 0.5, layer.ln2.numel()).to(layer.ln2.dtype))
    gpu = copy.deepcopy(cpu).to("cuda")
    gpu.device = torch.device("cuda")
    ge = _engine(gpu, "cuda", cfg, len(prompts))
    assert gpu.layers[0].attn.qkv_pf is not None and gpu.lm_head_p is not None, "fused decode chain not packed"
    x = torch.zeros((len(prompts), cfg.hidden_size), dtype=torch.bfloat16, device="cuda")
    assert gpu._rowscale_ok(x), "decode would not take the folded-norm fused chain"
    gp, gfirst, gd = _two_steps(ge, prompts)
    cp, cfirst, cd = _two_steps(_engine(cpu, "cpu", cfg, len(prompts)), prompts)
    scale = cp.abs().max().item()
    # prefill: bf16 GEMMs / attention vs the fp32-accumulating reference
    torch.testing.assert_close(gp, cp, atol=0.02 * scale, rtol=0.05)
    # the decode step fed the same tokens on both sides (rows whose first token agreed)
    same = [i for i, (a, b) in enumerate(zip(gfirst, cfirst)) if a == b]
    for i, (a, b) in enumerate(zip(gfirst, cfirst)):
        if a != b:  # only a near-tie of the reference may differ
            assert cp[i, a] >= cp[i].max() - 0.02 * scale, (i, a, b)
    assert same, "no row decoded the same token"
    torch.testing.assert_close(gd[same], cd[same], atol=0.02 * scale, rtol=0.05)
    # and the greedy decode token itself agrees (up to reference near-ties)
    for i in same:
        top = cd[i].topk(2)
        assert gd[i].argmax().item() == top.indices[0].item() or top.values[0] - top.values[1] < 0.02 * scale
