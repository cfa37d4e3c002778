#!/bin/bash
# 70B TP=8 rank: fewer launches per layer (in-launch gate_up SiLU, fused MLP with split gate_up,
# fused QKV -> attention at one kv head) re-measured on the round-5 chain
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=gpurun_out
for i in 1 2; do
  for cfg in "0 0 4" "1 0 4" "0 1 4" "0 0 1"; do
    set -- $cfg
    POLYKEY_GATE_UP_INLAUNCH=$1 POLYKEY_MLP_FUSED_SPLIT=$2 POLYKEY_QKV_MIN_KV=$3 timeout -k 10 200 \
      python3 tools/tp_solo.py --model llama3-70b --tp 8 --iters 30 | cut -c1-120 \
      | sed "s/^{/{\"gu_inlaunch\": $1, \"mlp_fused_split\": $2, \"qkv_min_kv\": $3, /" | tee -a $O/r5_launches.jsonl || exit 1
  done
done
