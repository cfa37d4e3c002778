"""Where the fused QKV -> decode attention launch spends its time (Llama-3-8B layer, 64 sequences):
per-workgroup wall-clock stamps from tools/lab/qa_stamps.hip (a stamped copy of
csrc/kernels/decode_fused.hip's kernel).  Prints the QKV phase, the hand-off point of every kv
head and the attention tiles' end times, next to event timings of the production launch and of
its two halves as separate launches.  Weights and K/V rotate over 4 layers (cold like a step)."""
import ctypes
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from polykey_service_amd.ops import attention as A  # noqa: E402
from polykey_service_amd.ops import gemm  # noqa: E402
from polykey_service_amd.ops import native  # noqa: E402
from polykey_service_amd.ops import reference as ref  # noqa: E402

B, NQ, NKV, D, BS, H = 64, 32, 8, 128, 32, 4096
N = (NQ + 2 * NKV) * D
L = 4


def pct(v, q):
    v = sorted(v)
    return v[min(len(v) - 1, int(q * len(v)))]


def main() -> None:
    ctx = int(os.environ.get("QA_CTX", "384"))
    lib = ctypes.CDLL(os.path.join(os.path.dirname(os.path.abspath(__file__)), "lab", "libqa_stamps.so"))
    d = "cuda"
    maxb = 512 // BS + 1
    nblk = B * maxb + 1
    g = torch.Generator().manual_seed(0)
    perm = torch.randperm(B * maxb, generator=g).to(torch.int32)  # scattered blocks, as after a while of serving
    bt = perm.view(B, maxb).to(d)
    ctxs = torch.full((B,), ctx, dtype=torch.int32)  # a bench wave: every sequence at the same position
    cl = ctxs.to(d)
    pos = (cl - 1)
    slots = (bt.gather(1, ((cl - 1) // BS).long()[:, None])[:, 0] * BS + (cl - 1) % BS).to(torch.int32)
    cs = ref.rope_cos_sin_cache(8192, D, 500000.0).to(d)
    layers = []
    for _ in range(L):
        w = (torch.randn(N, H, device=d) * 0.02).to(torch.bfloat16)
        layers.append((gemm.pack_weight(w), torch.randn(nblk, NKV, BS, D, device=d).to(torch.bfloat16),
                       torch.randn(nblk, NKV, D, BS, device=d).to(torch.bfloat16)))
    res = torch.randn(B, H, device=d).to(torch.bfloat16)
    wmeta = torch.empty((N, H), dtype=torch.bfloat16, device="meta")
    parts = gemm.residual_parts(None, res.clone(), torch.empty((H // gemm.PART_COLS) * B, device=d)).view(-1, B)
    rs = gemm.RowScale(parts, 1e-5)
    S = gemm.choose_split(N, H, B)
    ws = torch.empty(16 * B * N, dtype=torch.float32, device=d)
    flow = torch.zeros(gemm.FLOW_WORDS, dtype=torch.int32, device=d)
    po, pml = A.decode_workspace(B, NQ, maxb, BS, d)
    md = A.AttnMetadata(num_decode=B, num_prefill=0, num_prefill_tokens=0, max_prefill_q_len=0, slot_mapping=slots,
                        decode_block_tables=bt, decode_context_lens=cl, decode_part_o=po, decode_part_ml=pml,
                        decode_max_ctx=512)
    scale = 1 / D ** 0.5
    out = torch.empty(B, NQ * D, dtype=torch.bfloat16, device=d)
    grid = max(NKV * B, (N // 128) * S)
    st = torch.zeros(4 * grid, dtype=torch.int64, device=d)

    def stamped(i, pre=0):
        wp, kc, vc = layers[i % L]
        a = gemm.GemmArgs()
        a.partial, a.A, a.W = ws.data_ptr(), res.data_ptr(), wp.data_ptr()
        a.M, a.N, a.K, a.lda, a.ldo, a.S = B, N, H, H, N, S
        a.row_scale, a.nrm_parts, a.nrm_nparts, a.eps = 1, parts.data_ptr(), parts.numel() // B, 1e-5
        rc = lib.qa_stamped_launch(ctypes.byref(a), ctypes.c_void_p(out.data_ptr()), ctypes.c_void_p(pos.data_ptr()),
                                   ctypes.c_void_p(cs.data_ptr()), ctypes.c_void_p(slots.data_ptr()),
                                   ctypes.c_void_p(kc.data_ptr()), ctypes.c_void_p(vc.data_ptr()),
                                   ctypes.c_void_p(bt.data_ptr()), ctypes.c_void_p(cl.data_ptr()), NQ, NKV, BS, maxb,
                                   NQ * D, ctypes.c_float(scale), ctypes.c_void_p(flow.data_ptr()),
                                   ctypes.c_void_p(st.data_ptr()), pre, ctypes.c_void_p(native.stream_ptr()))
        assert rc == 0, rc

    def fused(i, s_=None):
        wp, kc, vc = layers[i % L]
        gemm.qkv_attn_fused(res, wp, rs, ws, pos, cs, kc, vc, md, scale, NQ, NKV, flow, S=s_)

    def qkv_only(i):
        wp, kc, vc = layers[i % L]
        gemm.linear_partial_rowscale(res, wmeta, ws, rs, S=S, packed=wp)

    def attn_only(i):
        wp, kc, vc = layers[i % L]
        A.paged_decode_from_qkv(gemm.Partial(ws, S, B, N), pos, cs, kc, vc, md, scale, NQ, NKV)

    def timeit(fn, n=40):
        for i in range(L):
            fn(i)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for i in range(n):
            fn(i)
        e1.record()
        torch.cuda.synchronize()
        return round(e0.elapsed_time(e1) * 1000 / n, 2)

    row = {"ctx_mean": float(ctxs.float().mean()), "S": S}
    for rep in range(3):
        row[f"fused_us_{rep}"] = timeit(fused)
    for name, fn in (("stamped_us", stamped), ("qkv_us", qkv_only), ("attn_us", attn_only)):
        try:
            row[name] = timeit(fn)
        except Exception as e:  # noqa: BLE001 - a lab: report and go on
            row[name] = f"error: {e}"
    print(json.dumps(row), flush=True)
    # stamps of a few single launches (the previous layer's launch drained: cold like a step)
    for rep in range(4):
        stamped(rep, pre=2 * (rep % 2))
        torch.cuda.synchronize()
        s = st.view(grid, 4).cpu().tolist()
        t0 = min(r[0] for r in s)
        us = lambda t: (t - t0) / 100.0  # 100 MHz
        n_qkv = (N // 128) * S
        qend = [us(r[1]) for r in s[:n_qkv]]
        # kv head of each QKV n-block (q heads by GQA group, then k, v heads)
        G = NQ // NKV

        def kvh(nb):
            return nb // G if nb < NQ else (nb - NQ if nb < NQ + NKV else nb - NQ - NKV)

        ready = [max(qend[b] for b in range(n_qkv) if kvh(b // S) == h) for h in range(NKV)]
        aend_plain = [us(r[2]) for b, r in enumerate(s) if b >= n_qkv]
        aend_q = [us(r[2]) for b, r in enumerate(s) if b < n_qkv]
        starts = [us(r[0]) for r in s]
        xcc = {}
        for r in s:
            xcc[r[3]] = xcc.get(r[3], 0) + 1
        print(json.dumps({
            "rep": rep, "pre": 2 * (rep % 2), "span_us": round(max(us(r[2]) for r in s), 2),
            "dispatch_last_start_us": round(max(starts), 2),
            "qkv_end_us": [round(pct(qend, q), 2) for q in (0.0, 0.5, 0.9, 1.0)],
            "kv_head_ready_us": [round(x, 2) for x in ready],
            "attn_end_us_plain_wgs": [round(pct(aend_plain, q), 2) for q in (0.0, 0.5, 0.9, 1.0)],
            "attn_end_us_qkv_wgs": [round(pct(aend_q, q), 2) for q in (0.0, 0.5, 0.9, 1.0)],
            "attn_dur_after_ready_us_plain": [round(pct([us(r[2]) - ready[b % NKV] for b, r in enumerate(s)
                                                         if b >= n_qkv], q), 2) for q in (0.0, 0.5, 0.9, 1.0)],
            "wgs_per_xcc": xcc}), flush=True)


if __name__ == "__main__":
    main()
