"""Decode-step time of ONE rank of a TP group at its real per-rank shapes, on one GPU, without
its peers: the model is built as rank 0 of a ``--tp`` group (Llama-3-70B TP=8: H 8192, 8 q / 1 kv
heads, gate_up 7168 x 8192, down 8192 x 3584, 16,128-row LM-head shard) and every collective is
replaced by its local part (``SoloAR``: the fused TP collective becomes the local slab sum +
residual add + norm parts; the logits all-gather a concatenation).  What it measures is the
per-rank GPU time of the decode chain minus the xGMI exchanges -- the part of a TP=8 step that
the one-GPU 8-rank rehearsal cannot show (its ranks share the CUs).  ``--tp 1`` times the full
single-GPU model the same way.

    python tools/tp_solo.py --model llama3-70b --tp 8 --batch 64 --ctx 384 [--layers 80]

One JSON line: ms per decode step (HIP graph replay, rotating nothing: the weights of a 70B shard
are 17.6 GB, far past the Infinity Cache) and the chain's kernels per layer.
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from polykey_service_amd.models import build_model, get_config  # noqa: E402
from polykey_service_amd.ops import attention as A  # noqa: E402
from polykey_service_amd.ops import gemm  # noqa: E402
from polykey_service_amd.parallel import comm  # noqa: E402
from polykey_service_amd.parallel.state import ParallelState, set_state  # noqa: E402


# SOLO_AR_NOOP=1: every collective does nothing (not even the local slab sum): times the GEMM side of
# the TP chain alone, chunked (POLYKEY_TP_DECODE_CHUNKS > 1) or not, like for like
NOOP = os.environ.get("SOLO_AR_NOOP") == "1"


class SoloAR:
    """The local half of every TP collective (no peers)."""

    def __init__(self, tp):
        self.tp = tp
        self.fused_blocks = 0

    def supports(self, x):
        return True

    def all_reduce(self, x, out=None, algo=0):
        return x if out is None or out is x else out.copy_(x)

    def supports_gather(self, x):
        return True

    def all_gather_last(self, x):
        return torch.cat([x] * self.tp, dim=-1)

    def supports_reduce_residual(self, M, N):
        return N % 1024 == 0

    def reduce_residual(self, pending, residual, parts):
        if NOOP:
            return parts.view(-1)[: (residual.shape[1] // 512) * residual.shape[0]].view(-1, residual.shape[0])
        return gemm.residual_parts(pending, residual, parts)

    # column-chunk collectives of the overlapped TP chain (models/llama.py _tp_row_collective)
    def nparts(self, M, N):
        return N // 512

    def chunks_ok(self, M, N, chunks):
        return NOOP and chunks > 1 and N % (1024 * chunks) == 0

    def reduce_residual_chunk(self, pending, residual, parts, chunk, chunks):
        pass  # SOLO_AR_NOOP: only the GEMM side of the chunked chain is timed

    def check(self):
        pass


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="llama3-70b")
    ap.add_argument("--tp", type=int, default=8)
    ap.add_argument("--layers", type=int, default=0)
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--ctx", type=int, default=384)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--eager", action="store_true", help="no graph (for per-kernel traces with launch gaps)")
    ap.add_argument("--car", choices=["solo", "loopback"], default="solo",
                    help="collectives: their local half (SoloAR) or the real kernels on local stand-in peers")
    ap.add_argument("--wide-min-tiles", type=int, default=None,
                    help="override models.llama.WIDE_MFMA_MIN_TILES (wide decode on the prefill MFMA GEMM)")
    a = ap.parse_args()
    if a.wide_min_tiles is not None:
        from polykey_service_amd.models import llama
        llama.WIDE_MFMA_MIN_TILES = a.wide_min_tiles
    cfg = get_config(a.model)
    if a.layers:
        import dataclasses
        cfg = dataclasses.replace(cfg, num_layers=a.layers)
    dev = torch.device("cuda:0")
    st = ParallelState(tp_size=a.tp, tp_rank=0, device=dev)
    if a.tp > 1:
        if a.car == "loopback":
            from polykey_service_amd.parallel.custom_ar import CustomAllReduce
            st.custom_ar = CustomAllReduce.loopback(0, a.tp, dev)
        else:
            st.custom_ar = SoloAR(a.tp)
    set_state(st)
    t0 = time.perf_counter()
    model = build_model(cfg, st, torch.bfloat16, dev).init_random(0)
    model.pack_decode_weights()
    torch.cuda.synchronize()
    init_s = time.perf_counter() - t0
    B, BS = a.batch, 32
    at = model.layers[0].attn
    maxb = (a.ctx + BS) // BS + 1
    nblk = B * maxb + 1
    kv = [(torch.zeros(nblk, at.nkv, BS, 128, dtype=torch.bfloat16, device=dev),
           torch.zeros(nblk, at.nkv, 128, BS, dtype=torch.bfloat16, device=dev)) for _ in model.layers]
    bt = torch.arange(B * maxb, dtype=torch.int32, device=dev).view(B, maxb)
    cl = torch.full((B,), a.ctx, dtype=torch.int32, device=dev)
    pos = cl - 1
    slots = bt[:, (a.ctx - 1) // BS] * BS + (a.ctx - 1) % BS
    po, pml = A.decode_workspace(B, at.nq, maxb, BS, dev, kv_heads=at.nkv)
    md = A.AttnMetadata(num_decode=B, num_prefill=0, num_prefill_tokens=0, max_prefill_q_len=0, slot_mapping=slots,
                        decode_block_tables=bt, decode_context_lens=cl, decode_part_o=po, decode_part_ml=pml,
                        decode_max_ctx=A._PART if a.ctx <= A._PART else 0)
    ids = torch.randint(0, cfg.vocab_size, (B,), dtype=torch.int32, device=dev)

    def step():
        h = model(ids, pos, md, kv)
        return model.compute_logits(h)

    with torch.inference_mode():
        for _ in range(2):
            step()
        torch.cuda.synchronize()
        fn = step
        if not a.eager:
            g = torch.cuda.CUDAGraph()
            s = torch.cuda.Stream()
            s.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(s):
                step()
            torch.cuda.current_stream().wait_stream(s)
            with torch.cuda.graph(g):
                step()
            fn = g.replay
        fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(a.iters):
            fn()
        e1.record()
        torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / a.iters
    gemm.check_fused()
    carried = None
    if a.car == "loopback" and getattr(model, "_flow_car", None) is not None:
        # the carried chain (kernels/car_gemm.hip) against the plain one on the same inputs: the
        # loopback peers make the values meaningless but deterministic -- they must match bit for bit
        with torch.inference_mode():
            model.carry_collectives = False
            ref = step().clone()
            model.carry_collectives = True
            got = step()
            torch.cuda.synchronize()
            model.carry_collectives = None
        carried = {"taken": True, "bit_identical": bool(torch.equal(ref, got))}
    if a.car == "loopback":
        assert st.custom_ar.error() == 0, "a loopback wait timed out"
    print(json.dumps({"model": a.model, "tp": a.tp, "layers": cfg.num_layers, "batch": B, "ctx": a.ctx,
                      "ms_per_step": round(ms, 3), "us_per_layer": round(ms * 1000 / cfg.num_layers, 2),
                      "graph": not a.eager, "wide_min_tiles": a.wide_min_tiles, "init_s": round(init_s, 1), "car": a.car, "carried": carried,
                      "mlp_fused": os.environ.get("POLYKEY_MLP_FUSED", "1"),
                      "qkv_attn_fused": os.environ.get("POLYKEY_QKV_ATTN_FUSED", "1"),
                      "env": {k: v for k, v in os.environ.items() if k.startswith("POLYKEY_")}}), flush=True)


if __name__ == "__main__":
    main()
