#!/bin/bash
# 70B TP=8 gate_up as 64-row n-blocks without a K split (POLYKEY_GATE_UP_KR1): test, A/B, profile
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/kernels/test_phases.py -k "gate_up" \
  > $O/r5_kr1_tests.log 2>&1; rc=$?; tail -2 $O/r5_kr1_tests.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  for k in 0 1; do
    POLYKEY_GATE_UP_KR1=$k timeout -k 10 200 python3 tools/tp_solo.py --model llama3-70b --tp 8 --iters 30 | cut -c1-130 \
      | sed "s/^{/{\"gate_up_kr1\": $k, /" | tee -a $O/r5_kr1.jsonl || exit 1
  done
done
cd /tmp && export TMPDIR=/tmp
POLYKEY_GATE_UP_KR1=1 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d /tmp/s70 -- python3 $R/tools/tp_solo.py --model llama3-70b \
  --tp 8 --iters 10 --eager > /tmp/s70.log 2>&1 || { tail -20 /tmp/s70.log; exit 1; }
python3 $R/tools/kgrid.py /tmp/s70 $R/$O/r5_70b_kgrid_kr1.md --per 13 > /dev/null
