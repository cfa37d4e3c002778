#!/bin/bash
# decode-fill threshold at small batches (8B: 8 kv heads; 70B TP=8: 1 kv head)
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=gpurun_out
for b in 8 16 32; do
  for f in 64 256; do
    POLYKEY_DECODE_FILL=$f timeout -k 10 200 python3 tools/tp_solo.py --model llama3-8b --tp 1 --batch $b --iters 30 | cut -c1-120 \
      | sed "s/^{/{\"fill\": $f, /" | tee -a $O/r5_fill_small.jsonl || exit 1
  done
done
for b in 16 32; do
  for f in 64 256; do
    POLYKEY_DECODE_FILL=$f timeout -k 10 200 python3 tools/tp_solo.py --model llama3-70b --tp 8 --batch $b --iters 30 | cut -c1-120 \
      | sed "s/^{/{\"fill\": $f, /" | tee -a $O/r5_fill_small.jsonl || exit 1
  done
done
