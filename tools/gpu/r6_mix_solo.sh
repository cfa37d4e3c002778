#!/bin/bash
# Mixtral decode step (graph replay, tools/tp_solo.py) with / without the fused QKV -> attention launch
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=gpurun_out
rm -f $O/r6_mix_solo.jsonl
for i in 1 2 3; do
  for f in 1 0; do
    POLYKEY_QKV_ATTN_FUSED=$f timeout -k 10 300 python3 tools/tp_solo.py --model mixtral-8x7b --tp 1 --batch 64 --ctx 384 --iters 20 \
      | cut -c1-160 | sed "s/^{/{\"fused\": $f, /" | tee -a $O/r6_mix_solo.jsonl || exit 1
  done
done
