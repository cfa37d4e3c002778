#!/bin/bash
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=gpurun_out
for i in 1 2; do
  for m in 1 2; do
    POLYKEY_HALF_SPLIT_MUL=$m timeout -k 10 200 python3 tools/tp_solo.py --model llama3-8b --tp 1 --iters 30 | cut -c1-120 \
      | sed "s/^{/{\"half_split_mul\": $m, /" | tee -a $O/r5_osplit.jsonl || exit 1
    POLYKEY_HALF_SPLIT_MUL=$m timeout -k 10 200 python3 tools/tp_solo.py --model llama3-70b --tp 8 --iters 30 | cut -c1-120 \
      | sed "s/^{/{\"half_split_mul\": $m, /" | tee -a $O/r5_osplit.jsonl || exit 1
  done
done
