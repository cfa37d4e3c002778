#!/bin/bash
# 70B TP=8 per-rank decode step with the real collective kernels on local stand-in peers
# (--car loopback), plain vs the GEMM-epilogue push (POLYKEY_TP_PUSH)
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=gpurun_out
timeout -k 10 120 python3 -u -m pytest -x -q --timeout 100 --timeout-method thread tests/parallel/test_custom_ar_gpu.py -k loopback > $O/r5_loopback_test.log 2>&1 || { tail -30 $O/r5_loopback_test.log; exit 1; }
tail -1 $O/r5_loopback_test.log
for i in 1 2; do
  for v in "solo 0" "loopback 0" "loopback 1"; do
    set -- $v
    POLYKEY_TP_PUSH=$2 timeout -k 10 200 python3 tools/tp_solo.py --model llama3-70b --tp 8 --iters 30 --car $1 | cut -c1-150 \
      | sed "s/^{/{\"push\": $2, /" | tee -a $O/r5_loopback.jsonl || exit 1
  done
done
