#!/bin/bash
# A/B: next projection's first weight MB read on a side stream during each TP decode collective
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=gpurun_out
for i in 1 2; do
  for mb in 0 16 48; do
    POLYKEY_TP_PREFETCH_MB=$mb timeout -k 10 200 python3 tools/tp_solo.py --model llama3-70b --tp 8 --iters 30 --car loopback | cut -c1-150 \
      | sed "s/^{/{\"prefetch_mb\": $mb, /" | tee -a $O/r5_prefetch.jsonl || exit 1
  done
done
