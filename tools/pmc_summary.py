"""Aggregate a ``rocprofv3 --pmc ... --output-format csv`` run into a per-kernel table.

Usage: python tools/pmc_summary.py <rocprof output dir> [out.md]

Per kernel: dispatches, total/avg time (from the counter rows' timestamps), and the summed
counters.  Derived columns (gfx94x formulas; ROCm 7.2 ships no gfx950 derived-counter XML, so
these are computed here explicitly):
  * MFMA util  = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 XCDs * 256 CUs * 4 SIMDs)
                 (GRBM_GUI_ACTIVE comes back summed over the 8 XCDs' GRBMs; with that
                 normalisation the hipBLASLt prefill GEMMs read ~80 %, consistent with their
                 FLOP-derived ~1.5 PF/s at the serialized-dispatch clock)
  * HBM read   = FETCH_SIZE (KiB) * 2 / time — gfx950 FETCH_SIZE reports half the bytes of wide
                 coalesced streaming reads (MI355X_MICROARCH.md §HBM); shown as TB/s.
  * SQ busy    = SQ_BUSY_CYCLES / GRBM_GUI_ACTIVE (per-SE average, a coarse occupancy proxy)
"""
import collections
import csv
import glob
import os
import sys

N_CU, N_SIMD, N_XCD = 256, 4, 8


def short(name: str) -> str:
    """Demangled signature → qualified name with template args, without the parameter list."""
    name = name.replace("(anonymous namespace)::", "")
    if name.startswith("void "):
        name = name[5:]
    depth = 0
    for i, ch in enumerate(name):
        if ch == "<":
            depth += 1
        elif ch == ">":
            depth -= 1
        elif ch == "(" and depth == 0:
            name = name[:i]
            break
    return name[:90]


def main(argv):
    root = argv[0]
    files = glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True)
    if not files:
        raise SystemExit(f"no counter_collection.csv under {root}")
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(set)
    tim = collections.defaultdict(dict)
    for f in files:
        with open(f, newline="") as fh:
            for r in csv.DictReader(fh):
                k = short(r.get("Kernel_Name", "?"))
                did = (f, r.get("Dispatch_Id"))
                agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
                disp[k].add(did)
                if "Start_Timestamp" in r and r.get("End_Timestamp"):
                    tim[k][did] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    rows = []
    for k, c in agg.items():
        t_ns = sum(tim[k].values())
        n = len(disp[k])
        gui = c.get("GRBM_GUI_ACTIVE", 0.0)
        mfma = c.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0) / (gui / N_XCD * N_CU * N_SIMD) if gui else 0.0
        hbm = c.get("FETCH_SIZE", 0.0) * 1024 * 2 / t_ns / 1e3 if t_ns else 0.0
        busy = c.get("SQ_BUSY_CYCLES", 0.0) / gui if gui else 0.0
        lds = c.get("SQ_LDS_BANK_CONFLICT", 0.0) / n if n else 0.0
        rows.append((t_ns, k, n, mfma, hbm, busy, lds))
    rows.sort(reverse=True)
    total = sum(r[0] for r in rows) or 1
    out = ["| kernel | calls | total ms | % | avg us | MFMA util | HBM rd TB/s (x2 corr.) | SQ busy/GUI | LDS bank confl/call |",
           "|---|---|---|---|---|---|---|---|---|"]
    for t_ns, k, n, mfma, hbm, busy, lds in rows[:40]:
        out.append(f"| `{k}` | {n} | {t_ns/1e6:.2f} | {100*t_ns/total:.1f} | {t_ns/max(n,1)/1e3:.1f} | "
                   f"{100*mfma:.1f}% | {hbm:.2f} | {busy:.2f} | {lds:.0f} |")
    # every collected counter, per call, for the top kernels
    names = sorted({c for k in agg for c in agg[k]})
    out += ["", "Raw counters per call:", "", "| kernel | " + " | ".join(names) + " |",
            "|---|" + "---|" * len(names)]
    for t_ns, k, n, *_ in rows[:8]:
        out.append(f"| `{k[:60]}` | " + " | ".join(f"{agg[k].get(c, 0.0) / max(n, 1):.4g}" for c in names) + " |")
    text = "\n".join(out) + "\n"
    if len(argv) > 1:
        with open(argv[1], "w") as fh:
            fh.write(text)
    print(text)


if __name__ == "__main__":
    main(sys.argv[1:])
