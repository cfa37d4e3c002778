"""Summarise a rocprofv3 ``--kernel-trace --stats --output-format csv`` directory:
top kernels by total time, with per-call averages.  Usage: kstats.py <dir> [out.md] [top]"""
import csv
import glob
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_summary import short  # noqa: E402


def main(argv):
    f = glob.glob(os.path.join(argv[0], "**", "*kernel_stats.csv"), recursive=True)[0]
    top = int(argv[2]) if len(argv) > 2 else 40
    rows = list(csv.DictReader(open(f)))
    tot = sum(float(r["TotalDurationNs"]) for r in rows) or 1.0
    out = [f"total GPU kernel time {tot / 1e6:.1f} ms", "",
           "| kernel | calls | total ms | % | avg us |", "|---|---|---|---|---|"]
    for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:top]:
        t = float(r["TotalDurationNs"])
        out.append(f"| `{short(r['Name'])}` | {r['Calls']} | {t / 1e6:.2f} | {100 * t / tot:.1f} | "
                   f"{float(r['AverageNs']) / 1e3:.1f} |")
    text = "\n".join(out) + "\n"
    if len(argv) > 1:
        open(argv[1], "w").write(text)
    print(text)


if __name__ == "__main__":
    main(sys.argv[1:])
