#!/bin/bash
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=gpurun_out
for i in 1 2; do
  for h in 0 1; do
    POLYKEY_GATE_UP_HALF=$h timeout -k 10 200 python3 tools/tp_solo.py --model llama3-70b --tp 8 --iters 30 --car loopback | cut -c1-150 \
      | sed "s/^{/{\"gate_up_half\": $h, /" | tee -a $O/r5_guhalf.jsonl || exit 1
  done
done
