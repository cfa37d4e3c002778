#!/bin/bash
# headline bench under a kernel trace + stats (per-kernel step breakdown of the current code)
set -o pipefail
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_r2e -- python3 $R/bench.py --steps 1 --warmup 1 > $R/gpurun_out/prof_r2e.log 2>&1
