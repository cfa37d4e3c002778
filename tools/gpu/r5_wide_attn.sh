#!/bin/bash
# 8-wave decode attention workgroups for launches of <= 128 workgroups (70B TP=8 rank)
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 240 --timeout-method thread \
  tests/kernels/test_phases.py -k "partition_merge" tests/kernels/test_attention.py > $O/r5_wa_tests.log 2>&1; rc=$?; tail -2 $O/r5_wa_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 tools/attn70_probe.py | cut -c1-100 | tee $O/r5_attn70_probe3.jsonl || exit 1
for i in 1 2; do
  for w in 0 1; do
    POLYKEY_DECODE_WIDE=$w timeout -k 10 200 python3 tools/tp_solo.py --model llama3-70b --tp 8 --iters 30 | cut -c1-120 \
      | sed "s/^{/{\"wide\": $w, /" | tee -a $O/r5_wide_attn.jsonl || exit 1
  done
done
