#!/bin/bash
# the driver's N=2 / N=4 runs put the 70B TP child at TP = 2 / 4: those per-rank shapes, solo
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=gpurun_out
for tp in 2 4; do
  timeout -k 10 300 python3 tools/tp_solo.py --model llama3-70b --tp $tp --iters 20 | cut -c1-200 | tee -a $O/r5_tp24.jsonl || exit 1
done
