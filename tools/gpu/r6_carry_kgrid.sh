#!/bin/bash
# per-(kernel, grid) profile of the 70B TP=8 rank on the loopback group, plain vs carried chain
set -o pipefail
R=$GRAFT_REPO_ROOT
O=gpurun_out
cd /tmp && export TMPDIR=/tmp
for c in 0 1; do
  rm -rf /tmp/lc$c
  POLYKEY_TP_CARRY=$c timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d /tmp/lc$c -- python3 $R/tools/tp_solo.py --model llama3-70b \
    --tp 8 --iters 10 --eager --car loopback > $R/$O/r6_carry_kgrid_$c.log 2>&1 || exit 1
  python3 $R/tools/kgrid.py /tmp/lc$c $R/$O/r6_carry_kgrid_$c.md --per 13 > /dev/null || exit 1
  head -16 $R/$O/r6_carry_kgrid_$c.md | cut -c1-200
done
