#!/bin/bash
# wide decode batches (8B TP=1, ctx 384): per-step time and per-kernel breakdown at 128 / 256 / 512 rows
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=gpurun_out
for b in 64 128 256 512; do
  timeout -k 10 200 python3 tools/tp_solo.py --model llama3-8b --tp 1 --batch $b --iters 20 | cut -c1-130 | tee -a $O/r5_wide.jsonl || exit 1
done
cd /tmp && export TMPDIR=/tmp
for b in 256 512; do
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d /tmp/w$b -- python3 $R/tools/tp_solo.py --model llama3-8b \
    --tp 1 --batch $b --iters 10 --eager > /tmp/w$b.log 2>&1 || { tail -20 /tmp/w$b.log; exit 1; }
  python3 $R/tools/kgrid.py /tmp/w$b $R/$O/r5_wide_${b}_kgrid.md --per 13 > /dev/null
done
