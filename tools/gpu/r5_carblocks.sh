#!/bin/bash
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=gpurun_out
for nb in 0 128 64; do
  POLYKEY_CAR_FUSED_BLOCKS=$nb timeout -k 10 120 python3 tools/car_probe.py | sed "s/^{/{\"fused_blocks\": $nb, /" | tee -a $O/r5_carblocks.jsonl || exit 1
done
for i in 1 2; do
  for nb in 0 128; do
    POLYKEY_CAR_FUSED_BLOCKS=$nb timeout -k 10 200 python3 tools/tp_solo.py --model llama3-70b --tp 8 --iters 30 --car loopback | cut -c1-150 \
      | sed "s/^{/{\"fused_blocks\": $nb, /" | tee -a $O/r5_carblocks.jsonl || exit 1
  done
done
