#!/bin/bash
# 8B per-rank decode step at 256 and 512 rows after the wide-decode change: per-(kernel, grid) profile (eager)
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
cd /tmp && export TMPDIR=/tmp
for b in 256 512; do
  rm -rf /tmp/wk$b
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d /tmp/wk$b -- python3 $R/tools/tp_solo.py --model llama3-8b --tp 1 --batch $b --ctx 384 --iters 10 --eager > $O/r6_wide_kgrid_$b.log 2>&1 || exit 1
  python3 $R/tools/kgrid.py /tmp/wk$b $O/r6_wide_${b}_kgrid.md --per 13 > /dev/null || exit 1
  head -22 $O/r6_wide_${b}_kgrid.md | cut -c1-160
done
