#!/bin/bash
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 240 --timeout-method thread \
  tests/e2e/test_engine_gpu.py -k "large_decode" > $O/r5_qw_tests.log 2>&1; rc=$?; tail -2 $O/r5_qw_tests.log; [ $rc -eq 0 ] || exit $rc
for b in 512 256; do
  for t in 384 1024 192; do
    POLYKEY_QKV_SKINNY_MAX_M=$t timeout -k 10 200 python3 tools/tp_solo.py --model llama3-8b --tp 1 --batch $b --iters 20 | cut -c1-130 \
      | sed "s/^{/{\"qkv_max_m\": $t, /" | tee -a $O/r5_qkv_wide.jsonl || exit 1
  done
done
