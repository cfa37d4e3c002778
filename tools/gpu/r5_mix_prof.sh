#!/bin/bash
# Mixtral bench wave under a kernel trace -> step breakdown (the trace itself stays on the box)
set -o pipefail
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 500 rocprofv3 --kernel-trace --output-format csv -d /tmp/prof_mix5 -- python3 $R/bench.py --model mixtral-8x7b --steps 1 --warmup 1 > $R/gpurun_out/prof_mix5.log 2>&1 \
  && python3 $R/tools/step_breakdown.py /tmp/prof_mix5 $R/gpurun_out/r5_mixtral_step_breakdown.md > /dev/null
