#!/bin/bash
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=gpurun_out
for i in 1 2; do
  for d in 1 2; do
    POLYKEY_HALF_SPLIT_DIV=$d timeout -k 10 200 python3 tools/tp_solo.py --model llama3-70b --tp 8 --iters 30 | cut -c1-110 \
      | sed "s/^{/{\"half_split_div\": $d, /" | tee -a $O/r5_osplit2.jsonl || exit 1
    POLYKEY_HALF_SPLIT_DIV=$d timeout -k 10 200 python3 tools/tp_solo.py --model llama3-8b --tp 1 --iters 30 | cut -c1-110 \
      | sed "s/^{/{\"half_split_div\": $d, /" | tee -a $O/r5_osplit2.jsonl || exit 1
  done
done
