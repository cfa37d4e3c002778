#!/bin/bash
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=gpurun_out
for i in 1 2; do
  for mb in 160 100; do
    POLYKEY_NT_MIN_MB=$mb timeout -k 10 200 python3 tools/tp_solo.py --model llama3-70b --tp 8 --iters 30 | cut -c1-130 \
      | sed "s/^{/{\"nt_min_mb\": $mb, /" | tee -a $O/r5_nt.jsonl || exit 1
  done
done
