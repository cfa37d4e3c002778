"""Merge a rocprofv3 kernel trace and memory-copy trace of the steady-state window and report
what sits in the GPU's idle gaps (copies, or nothing = host-bound).
Usage: trace_timeline.py <rocprof csv dir> [tail_fraction=0.1]"""
import csv
import glob
import os
import sys


def load(root, pat):
    fs = glob.glob(os.path.join(root, "**", pat), recursive=True)
    return list(csv.DictReader(open(fs[0]))) if fs else []


def main(argv):
    root = argv[0]
    frac = float(argv[1]) if len(argv) > 1 else 0.1
    ks = sorted(load(root, "*kernel_trace.csv"), key=lambda r: int(r["Start_Timestamp"]))
    cps = load(root, "*memory_copy_trace.csv")
    ks = ks[int(len(ks) * (1 - frac)):]
    t0, t1 = int(ks[0]["Start_Timestamp"]), int(ks[-1]["End_Timestamp"])
    cps = [c for c in cps if t0 <= int(c["Start_Timestamp"]) <= t1]
    kinds = {}
    for c in cps:
        key = c.get("Direction", c.get("Kind", "?"))
        d = int(c["End_Timestamp"]) - int(c["Start_Timestamp"])
        n, tot, b = kinds.get(key, (0, 0, 0))
        kinds[key] = (n + 1, tot + d, b + int(c.get("Size", c.get("Bytes", 0)) or 0))
    print(f"window {(t1 - t0) / 1e6:.1f} ms, {len(ks)} kernels, {len(cps)} copies")
    for k, (n, tot, b) in kinds.items():
        print(f"  copy {k}: {n} x avg {tot / n / 1e3:.1f} us, avg {b / n / 1e3:.1f} KB")
    gaps = []
    for a, b in zip(ks, ks[1:]):
        ga, gb = int(a["End_Timestamp"]), int(b["Start_Timestamp"])
        if gb - ga > 20000:
            inside = [c for c in cps if int(c["End_Timestamp"]) > ga and int(c["Start_Timestamp"]) < gb]
            cov = sum(min(gb, int(c["End_Timestamp"])) - max(ga, int(c["Start_Timestamp"])) for c in inside)
            gaps.append((gb - ga, cov, len(inside), a["Kernel_Name"][:40], b["Kernel_Name"][:40]))
    tot = sum(g[0] for g in gaps)
    cov = sum(g[1] for g in gaps)
    print(f"{len(gaps)} gaps > 20 us: {tot / 1e6:.2f} ms total, copies active during {cov / 1e6:.2f} ms of it")
    from collections import Counter
    c = Counter((g[3], g[4]) for g in gaps)
    for (a, b), n in c.most_common(6):
        sel = [g for g in gaps if (g[3], g[4]) == (a, b)]
        print(f"  {n:4d} x {sum(g[0] for g in sel) / n / 1e3:7.1f} us  after {a!r} before {b!r}  "
              f"(copies in gap: {sum(g[2] for g in sel) / n:.1f})")


if __name__ == "__main__":
    main(sys.argv[1:])
