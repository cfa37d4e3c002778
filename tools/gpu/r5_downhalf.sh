#!/bin/bash
# A/B: 8B decode down projection as 64-row tiles at half the split (POLYKEY_DOWN_HALF)
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=gpurun_out
POLYKEY_DOWN_HALF=1 timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/kernels/test_phases.py tests/kernels/test_gemm_skinny.py -m gpu > $O/r5_downhalf_tests.log 2>&1 || exit 1
tail -1 $O/r5_downhalf_tests.log
for i in 1 2; do
  for d in 0 1; do
    POLYKEY_DOWN_HALF=$d timeout -k 10 200 python3 tools/tp_solo.py --model llama3-8b --tp 1 --iters 30 | cut -c1-110 \
      | sed "s/^{/{\"down_half\": $d, /" | tee -a $O/r5_downhalf.jsonl || exit 1
  done
done
