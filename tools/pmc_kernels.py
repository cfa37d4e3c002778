"""Per-kernel average of every PMC counter in a rocprofv3 --pmc CSV (one row per kernel name).
Usage: pmc_kernels.py <counter_collection.csv> [name filter]"""
import collections
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
flt = sys.argv[2] if len(sys.argv) > 2 else ""
agg = collections.defaultdict(lambda: collections.defaultdict(float))
cnt = collections.Counter()
for r in rows:
    k = r["Kernel_Name"][:70]
    if flt not in k:
        continue
    agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
    cnt[(k, r["Counter_Name"])] += 1
for k, v in agg.items():
    n = max(cnt[(k, c)] for c in v)
    print(f"{k}  (dispatches {n})")
    print("   " + "  ".join(f"{c}={x / n:.3g}" for c, x in sorted(v.items())))
