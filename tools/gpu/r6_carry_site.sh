#!/bin/bash
# per-site carry A/B (70B TP=8 rank on the loopback group, graph replay): plain, gate_up only, both
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=gpurun_out
for i in 1 2; do
  for c in 0 gate_up 1; do
    POLYKEY_TP_CARRY=$c timeout -k 10 200 python3 tools/tp_solo.py --model llama3-70b --tp 8 --iters 30 --car loopback \
      | cut -c1-260 | sed "s/^{/{\"carry\": \"$c\", /" | tee -a $O/r6_carry_site.jsonl || exit 1
  done
done
