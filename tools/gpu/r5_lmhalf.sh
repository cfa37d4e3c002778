#!/bin/bash
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=gpurun_out
POLYKEY_LINEAR_HALF=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/kernels/test_gemm_skinny.py \
  tests/parallel/test_tp_chain_gpu.py > $O/r5_lmh_tests.log 2>&1; rc=$?; tail -2 $O/r5_lmh_tests.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  for h in 0 1; do
    POLYKEY_LINEAR_HALF=$h timeout -k 10 200 python3 tools/tp_solo.py --model llama3-70b --tp 8 --iters 30 | cut -c1-110 \
      | sed "s/^{/{\"linear_half\": $h, /" | tee -a $O/r5_lmhalf.jsonl || exit 1
  done
done
