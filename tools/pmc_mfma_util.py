"""MFMA utilisation table from rocprofv3 --pmc CSVs (SQ_VALU_MFMA_BUSY_CYCLES summed over the
1024 SIMDs, GRBM_GUI_ACTIVE summed over the 8 XCDs of an MI355X):
    util = MFMA_BUSY / (GRBM_GUI_ACTIVE / 8 * 1024)
Usage: pmc_mfma_util.py <csv> [<csv> ...] [--filter name]"""
import collections
import csv
import sys

args = [a for a in sys.argv[1:] if not a.startswith("--")]
flt = sys.argv[sys.argv.index("--filter") + 1] if "--filter" in sys.argv else ""
if flt in args:
    args.remove(flt)
print("| kernel | dispatches | MFMA busy | VALU active / wave-cycles | LDS active / wave-cycles | wait any / wave-cycles | LDS bank-conflict cycles |")
print("|---|---|---|---|---|---|---|")
for path in args:
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    n = collections.Counter()
    for r in csv.DictReader(open(path)):
        k = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0][:60]
        if flt and flt not in k:
            continue
        agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
        if r["Counter_Name"] == "GRBM_GUI_ACTIVE":
            n[k] += 1
    for k, v in agg.items():
        util = v["SQ_VALU_MFMA_BUSY_CYCLES"] / (v["GRBM_GUI_ACTIVE"] / 8 * 1024) if v["GRBM_GUI_ACTIVE"] else 0
        wc = v["SQ_WAVE_CYCLES"] or 1
        print(f"| `{k}` | {n[k]} | {100 * util:.1f} % | {100 * v['SQ_ACTIVE_INST_VALU'] / wc:.1f} % | "
              f"{100 * v['SQ_ACTIVE_INST_LDS'] / wc:.1f} % | {100 * v['SQ_WAIT_ANY'] / wc:.1f} % | "
              f"{v['SQ_LDS_BANK_CONFLICT'] / max(n[k], 1):.3g} |")
