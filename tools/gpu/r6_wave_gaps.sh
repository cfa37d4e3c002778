#!/bin/bash
# idle time inside the headline bench wave: kernel trace of one timed wave, gaps by position
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
cd /tmp && export TMPDIR=/tmp
rm -rf /tmp/wg
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d /tmp/wg -- python3 $R/bench.py --steps 1 --warmup 1 > $O/r6_wave_gaps_bench.log 2>&1 || { tail -20 $O/r6_wave_gaps_bench.log; exit 1; }
python3 $R/tools/wave_gaps.py /tmp/wg 10 $O/r6_wave_gaps.md > /dev/null || exit 1
python3 $R/tools/step_breakdown.py /tmp/wg $O/r6_step_breakdown.md > /dev/null || exit 1
head -40 $O/r6_wave_gaps.md
head -20 $O/r6_step_breakdown.md
