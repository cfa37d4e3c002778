#!/bin/bash
# 8B graph-captured decode step (tools/tp_solo.py --tp 1): o-projection residual update in the O
# launch (last split of each 64-row n-block) vs o slabs + residual_parts, alternating
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
rm -f gpurun_out/ab2_solo.jsonl
for i in 1 2; do
  for v in 0 1; do
    POLYKEY_AB_O_INLAUNCH=$v timeout -k 10 300 python -u tools/tp_solo.py --model llama3-8b --tp 1 --iters 20 \
      > gpurun_out/ab2_solo_$v.log 2>&1 || { tail -20 gpurun_out/ab2_solo_$v.log; exit 1; }
    echo "{\"o_inlaunch\": $v, \"line\": $(tail -1 gpurun_out/ab2_solo_$v.log)}" | tee -a gpurun_out/ab2_solo.jsonl
  done
done
