#!/bin/bash
# decode GEMM tiles with 4 weight k-steps in flight (variant build) vs 2: correctness, per-rank step
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=gpurun_out
V=$R/tools/lab/libpk_kernels_wdepth4.so
POLYKEY_LIB_LIBPK_KERNELS=$V timeout -k 10 400 python -u -m pytest -x -q --timeout 240 --timeout-method thread \
  tests/kernels/test_gemm_skinny.py tests/kernels/test_phases.py > $O/r5_wd_tests.log 2>&1; rc=$?; tail -2 $O/r5_wd_tests.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  for v in base wd4; do
    if [ $v = wd4 ]; then export POLYKEY_LIB_LIBPK_KERNELS=$V; else unset POLYKEY_LIB_LIBPK_KERNELS; fi
    timeout -k 10 200 python3 tools/tp_solo.py --model llama3-70b --tp 8 --iters 30 | cut -c1-120 | sed "s/^{/{\"lib\": \"$v\", /" | tee -a $O/r5_wdepth.jsonl || exit 1
    timeout -k 10 200 python3 tools/tp_solo.py --model llama3-8b --tp 1 --iters 30 | cut -c1-120 | sed "s/^{/{\"lib\": \"$v\", /" | tee -a $O/r5_wdepth.jsonl || exit 1
  done
done
