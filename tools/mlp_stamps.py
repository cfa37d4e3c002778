"""Where the fused decode MLP launch spends its time (Llama-3-8B layer, 64 rows): per-workgroup
wall-clock stamps from tools/lab/qa_stamps.hip (a stamped copy of gemm_skinny.hip
mlp_fused_kernel): gate_up tile ends, each down K-slice's hand-off point, down tile ends, next
to event timings of the production launch and of gate_up / down as separate launches.  Weights
rotate over 4 layers (cold like a step)."""
import ctypes
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from polykey_service_amd.ops import gemm  # noqa: E402
from polykey_service_amd.ops import native  # noqa: E402

M, H, I = 64, 4096, 14336
L = 4


def pct(v, q):
    v = sorted(v)
    return v[min(len(v) - 1, int(q * len(v)))]


def main() -> None:
    lib = ctypes.CDLL(os.path.join(os.path.dirname(os.path.abspath(__file__)), "lab", "libqa_stamps.so"))
    d = "cuda"
    layers = []
    for _ in range(L):
        gu = (torch.randn(2 * I, H, device=d) * 0.02).to(torch.bfloat16)
        dn = (torch.randn(H, I, device=d) * 0.02).to(torch.bfloat16)
        layers.append((gemm.pack_weight(gu), gemm.pack_weight(dn)))
        del gu, dn
    x = torch.randn(M, H, device=d).to(torch.bfloat16)
    parts = gemm.residual_parts(None, x.clone(), torch.empty((H // gemm.PART_COLS) * M, device=d)).view(-1, M)
    rs = gemm.RowScale(parts, 1e-5)
    S = gemm.choose_split(H, I, M)
    ws = torch.empty(S * M * H, dtype=torch.float32, device=d)
    flow = torch.zeros(gemm.FLOW_WORDS, dtype=torch.int32, device=d)
    h = torch.empty(M, I, dtype=torch.bfloat16, device=d)
    dkr = 1 if (H // 128) * S < 192 else 2
    n_gu, n_dn = (2 * I) // 128, (H // (64 * dkr)) * S
    grid = max(n_gu, n_dn)
    st = torch.zeros(4 * grid, dtype=torch.int64, device=d)
    gmeta = torch.empty((2 * I, H), dtype=torch.bfloat16, device="meta")
    dmeta = torch.empty((H, I), dtype=torch.bfloat16, device="meta")

    def stamped(i):
        gp, dp = layers[i % L]
        gu = gemm.GemmArgs()
        gu.out, gu.A, gu.W = h.data_ptr(), x.data_ptr(), gp.data_ptr()
        gu.M, gu.N, gu.K, gu.lda, gu.ldo, gu.S = M, 2 * I, H, H, I, 1
        gu.row_scale, gu.nrm_parts, gu.nrm_nparts, gu.eps = 1, parts.data_ptr(), parts.shape[0], 1e-5
        dn = gemm.GemmArgs()
        dn.partial, dn.A, dn.W = ws.data_ptr(), h.data_ptr(), dp.data_ptr()
        dn.M, dn.N, dn.K, dn.lda, dn.ldo, dn.S = M, H, I, I, H, S
        rc = lib.mlp_stamped_launch(ctypes.byref(gu), ctypes.byref(dn), ctypes.c_void_p(flow.data_ptr()),
                                    ctypes.c_void_p(st.data_ptr()), ctypes.c_void_p(native.stream_ptr()))
        assert rc == 0, rc

    def fused(i):
        gp, dp = layers[i % L]
        gemm.mlp_fused(x, gp, dp, rs, ws, flow)

    def gate_up_only(i):
        gp, dp = layers[i % L]
        gemm.linear_silu(x, gmeta, packed=gp, rowscale=rs)

    def down_only(i):
        gp, dp = layers[i % L]
        gemm.linear_down(h, dmeta, ws, dp)

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

    row = {"S_down": S, "down_kr": dkr, "n_gu": n_gu, "n_dn": n_dn}
    for rep in range(3):
        row[f"fused_us_{rep}"] = timeit(fused, 60)
    for name, fn in (("stamped_us", stamped), ("gate_up_us", gate_up_only),
                     ("down_us", down_only)):
        try:
            row[name] = timeit(fn)
        except Exception as e:  # noqa: BLE001 - a lab: report and go on
            row[name] = f"error: {e}"
    print(json.dumps(row), flush=True)
    kslice = I // S  # h columns per down K slice; gate_up n-block nb writes h columns [64 nb, 64 nb + 64)
    for rep in range(3):
        stamped(rep)
        torch.cuda.synchronize()
        s = st.view(grid, 4).cpu().tolist()
        t0 = min(r[0] for r in s)
        us = lambda t: (t - t0) / 100.0
        gend = [us(r[1]) for r in s[:n_gu]]
        ready = [max(gend[nb] for nb in range(n_gu) if (64 * nb) // kslice == sl) for sl in range(S)]
        dend = [us(r[2]) for r in s[:n_dn]]
        dslice = [b % S for b in range(n_dn)]
        print(json.dumps({
            "rep": rep, "span_us": round(max(us(r[2]) for r in s), 2),
            "starts_us": [round(pct([us(r[0]) for r in s], q), 2) for q in (0.0, 0.5, 1.0)],
            "gate_up_end_us": [round(pct(gend, q), 2) for q in (0.0, 0.1, 0.5, 0.9, 1.0)],
            "slice_ready_us": [round(x, 2) for x in ready],
            "down_end_us": [round(pct(dend, q), 2) for q in (0.0, 0.1, 0.5, 0.9, 1.0)],
            "down_dur_after_ready_us": [round(pct([dend[b] - ready[dslice[b]] for b in range(n_dn)], q), 2)
                                        for q in (0.0, 0.5, 0.9, 1.0)]}), flush=True)


if __name__ == "__main__":
    main()
