"""Per-(kernel, grid) statistics from a rocprofv3 ``--kernel-trace --output-format csv`` directory:
the same kernel template launched for different projections (QKV vs gate_up, O vs down) has
different grids, so this splits what kstats.py lumps together.  Optionally only the last
``--tail`` dispatches (the timed iterations, after warm-up / weight init).

    python tools/kgrid.py <dir> [out.md] [--tail N] [--per STEPS]
"""
import argparse
import csv
import glob
import os
import sys
from collections import defaultdict

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_summary import short  # noqa: E402


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("out", nargs="?")
    ap.add_argument("--tail", type=int, default=0, help="only the last N dispatches")
    ap.add_argument("--per", type=int, default=0, help="divide totals by this many steps (us per step)")
    ap.add_argument("--top", type=int, default=30)
    a = ap.parse_args(argv)
    f = glob.glob(os.path.join(a.dir, "**", "*kernel_trace.csv"), recursive=True)[0]
    rows = list(csv.DictReader(open(f)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    if a.tail:
        rows = rows[-a.tail:]
    agg = defaultdict(list)
    for r in rows:
        grid = r.get("Grid_Size") or f"{r.get('Grid_Size_X')}x{r.get('Grid_Size_Y')}x{r.get('Grid_Size_Z')}"
        wg = r.get("Workgroup_Size") or r.get("Workgroup_Size_X")
        agg[(short(r["Kernel_Name"]), grid, wg)].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    tot = sum(sum(v) for v in agg.values()) or 1
    span = (int(rows[-1]["End_Timestamp"]) - int(rows[0]["Start_Timestamp"])) if rows else 0
    out = [f"{len(rows)} dispatches, kernel time {tot / 1e6:.2f} ms, span {span / 1e6:.2f} ms", "",
           "| kernel | grid | wg | calls | avg us | min us | total ms | % |" + (" us/step |" if a.per else ""),
           "|---|---|---|---|---|---|---|---|" + ("---|" if a.per else "")]
    for (k, g, w), v in sorted(agg.items(), key=lambda kv: -sum(kv[1]))[:a.top]:
        line = (f"| `{k}` | {g} | {w} | {len(v)} | {sum(v) / len(v) / 1e3:.1f} | {min(v) / 1e3:.1f} | "
                f"{sum(v) / 1e6:.2f} | {100 * sum(v) / tot:.1f} |")
        if a.per:
            line += f" {sum(v) / a.per / 1e3:.1f} |"
        out.append(line)
    text = "\n".join(out) + "\n"
    if a.out:
        open(a.out, "w").write(text)
    print(text)


if __name__ == "__main__":
    main()
