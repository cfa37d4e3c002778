#!/bin/bash
# WRITE_SIZE of the fused decode attention: V^T-row cache stores (old) vs fragment-native V (new)
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
for L in old new; do
  timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE GRBM_GUI_ACTIVE --output-format csv -d $R/gpurun_out/pmc_w_$L -- python3 $R/tools/attn_layout_lab.py --libs $L --ctx 384 --iters 20 --rounds 1 > $R/gpurun_out/pmc_w_$L.log 2>&1 || exit 1
done
cd $R
python3 - <<'PY'
import csv, glob, collections
for L in ("old", "new"):
    f = glob.glob(f"gpurun_out/pmc_w_{L}/**/*counter_collection.csv", recursive=True)[0]
    acc = collections.defaultdict(list)
    for r in csv.DictReader(open(f)):
        if r["Counter_Name"] == "WRITE_SIZE" and "paged_decode_kernel" in r["Kernel_Name"]:
            acc["qkv" if "true" in r["Kernel_Name"] else "q"].append(float(r["Counter_Value"]))
    for k, v in acc.items():
        print(f"{L} {k}: WRITE_SIZE {sum(v) / len(v):.0f} KB per launch over {len(v)} launches")
PY
