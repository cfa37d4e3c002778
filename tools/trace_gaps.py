"""Steady-state GPU busy fraction and inter-kernel gaps from a rocprofv3 kernel trace.
Usage: trace_gaps.py <rocprof csv dir> [tail_fraction=0.2]"""
import csv
import glob
import os
import sys


def main(argv):
    f = glob.glob(os.path.join(argv[0], "**", "*kernel_trace.csv"), recursive=True)[0]
    frac = float(argv[1]) if len(argv) > 1 else 0.2
    rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
    sub = rows[int(len(rows) * (1 - frac)):]
    t0, t1 = int(sub[0]["Start_Timestamp"]), int(sub[-1]["End_Timestamp"])
    busy = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in sub)
    gaps = sorted(int(b["Start_Timestamp"]) - int(a["End_Timestamp"]) for a, b in zip(sub, sub[1:]))
    big = [g for g in gaps if g > 20000]
    print(f"window: wall {(t1 - t0) / 1e6:.1f} ms, kernel busy {busy / 1e6:.1f} ms ({100 * busy / (t1 - t0):.1f}%), "
          f"{len(sub)} dispatches")
    print(f"gaps: p50 {gaps[len(gaps) // 2] / 1e3:.1f} us, p90 {gaps[int(len(gaps) * .9)] / 1e3:.1f} us, "
          f"{len(big)} gaps > 20 us summing {sum(big) / 1e6:.1f} ms (mean {sum(big) / max(len(big), 1) / 1e3:.0f} us)")


if __name__ == "__main__":
    main(sys.argv[1:])
