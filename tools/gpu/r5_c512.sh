#!/bin/bash
# wide decode batches after restricting the half-split QKV to single-tile batches
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=gpurun_out
for b in 256 512; do
  timeout -k 10 200 python3 tools/tp_solo.py --model llama3-8b --tp 1 --batch $b --iters 20 | cut -c1-120 | tee -a $O/r5_c512.jsonl || exit 1
done
for c in 512 256; do
  timeout -k 10 400 python -u bench.py --steps 2 --warmup 1 --concurrency $c > $O/c_$c.log 2>&1 || { tail -20 $O/c_$c.log; exit 1; }
  grep '^{"metric"' $O/c_$c.log | tee -a $O/r5_c512.jsonl | cut -c1-200
done
