#!/bin/bash
# 70B TP=1 (packed weights, one GPU): the fused decode launches on / off, alternating
set -o pipefail
for cfg in "0 0" "1 1" "1 0" "0 1"; do
  set -- $cfg
  POLYKEY_MLP_FUSED=$1 POLYKEY_QKV_ATTN_FUSED=$2 timeout -k 10 400 python bench.py --model llama3-70b --steps 1 --warmup 1 \
    > gpurun_out/b70_$1$2.json 2> gpurun_out/b70_$1$2.err || exit 1
  python -c "import json,sys; d=json.load(open('gpurun_out/b70_$1$2.json')); print('mlp=$1 qkv=$2', d['value'], d['ms_per_step'])"
done
