#!/bin/bash
# the 8-wave prefill GEMM (variant 4) on buffer_load ... lds staging: tests, then A/B against the 4-wave kernel
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=gpurun_out
timeout -k 10 300 python -u -m pytest tests/kernels/test_gemm_prefill.py -x -q --timeout 120 --timeout-method thread > $O/r6_pdeep_test.log 2>&1
rc=$?; tail -3 $O/r6_pdeep_test.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 tools/prefill_gemm_ab.py 4 6 | tee $O/r6_pdeep_ab.txt
