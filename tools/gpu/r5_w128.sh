#!/bin/bash
set -o pipefail
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d /tmp/w128 -- python3 $R/tools/tp_solo.py --model llama3-8b \
  --tp 1 --batch 128 --iters 10 --eager > /tmp/w128.log 2>&1 || { tail -20 /tmp/w128.log; exit 1; }
python3 $R/tools/kgrid.py /tmp/w128 $R/gpurun_out/r5_wide_128_kgrid.md --per 13 > /dev/null
