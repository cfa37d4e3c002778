#!/bin/bash
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=gpurun_out
PYTHONFAULTHANDLER=1 timeout -k 10 700 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/parallel/test_tp8_shapes_gpu.py tests/parallel/test_tp_gpu.py tests/parallel/test_tp_chain_gpu.py \
  > $O/r5_tp2_tests.log 2>&1; rc=$?; tail -3 $O/r5_tp2_tests.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  for c in 1 2 4; do
    SOLO_AR_NOOP=1 POLYKEY_TP_DECODE_CHUNKS=$c timeout -k 10 200 python3 tools/tp_solo.py --model llama3-70b --tp 8 \
      --iters 30 | cut -c1-160 | sed "s/^{/{\"chunks\": $c, /" | tee -a $O/r5_tp_chunks.jsonl || exit 1
  done
done
