#!/bin/bash
# 70B per-rank decode step at TP = 2 / 4 with the real collective kernels (loopback group)
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=gpurun_out
for tp in 2 4; do
  for c in solo loopback; do
    timeout -k 10 300 python3 tools/tp_solo.py --model llama3-70b --tp $tp --iters 20 --car $c | cut -c1-160 | tee -a $O/r5_tp24_loop.jsonl || exit 1
  done
done
