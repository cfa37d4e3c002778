#!/bin/bash
# round-3 headline bench under a kernel trace + stats, and the 256-client variant
set -o pipefail
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
for c in ${CONC:-64 256}; do
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_r3_c$c -- \
    python3 $R/bench.py --steps 1 --warmup 1 --concurrency $c > $R/gpurun_out/prof_r3_c$c.log 2>&1 || exit 1
  cd $R
  python3 tools/step_breakdown.py gpurun_out/prof_r3_c$c gpurun_out/r3_8b_c${c}_step_breakdown.md || exit 1
  find gpurun_out/prof_r3_c$c -name '*kernel_stats.csv' -exec cp {} gpurun_out/r3_8b_c${c}_kernel_stats.csv \;
  find gpurun_out/prof_r3_c$c -name '*kernel_trace.csv' -delete
  head -25 gpurun_out/r3_8b_c${c}_step_breakdown.md
  cd /tmp
done
