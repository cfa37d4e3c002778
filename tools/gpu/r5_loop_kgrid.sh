#!/bin/bash
# per-(kernel, grid) profile of the 70B TP=8 rank with the real collective kernels (loopback group)
set -o pipefail
R=$GRAFT_REPO_ROOT
O=gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d /tmp/l70 -- python3 $R/tools/tp_solo.py --model llama3-70b \
  --tp 8 --iters 10 --eager --car loopback > $R/$O/r5_loop_kgrid.log 2>&1 || exit 1
python3 $R/tools/kgrid.py /tmp/l70 $R/$O/r5_70b_tp8_loopback_kgrid.md --per 13 > /dev/null
