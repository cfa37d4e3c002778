#!/bin/bash
# headline bench under a kernel trace + stats (per-kernel step breakdown of the current code)
set -o pipefail
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_r2g -- python3 $R/bench.py --steps 1 --warmup 1 > $R/gpurun_out/prof_r2g.log 2>&1
rc=$?
cd $R
# kernel trace csv is large: keep only what step_breakdown needs plus the stats
python3 tools/step_breakdown.py gpurun_out/prof_r2g gpurun_out/r2g_8b_bench_step_breakdown.md || exit 1
find gpurun_out/prof_r2g -name '*kernel_stats.csv' -exec cp {} gpurun_out/r2g_8b_bench_kernel_stats.csv \;
find gpurun_out/prof_r2g -name '*kernel_trace.csv' -delete
exit $rc
