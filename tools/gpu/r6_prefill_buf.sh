#!/bin/bash
# prefill GEMM: buffer_load ... lds staging (variants 8 / 9) vs global_load_lds (6 / 7): tests, then same-process A/B
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=gpurun_out
timeout -k 10 300 python -u -m pytest tests/kernels/test_gemm_prefill.py -x -q --timeout 120 --timeout-method thread > $O/r6_pbuf_test.log 2>&1
rc=$?; tail -3 $O/r6_pbuf_test.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 tools/prefill_gemm_ab.py 6 8 | tee $O/r6_pbuf_ab.txt
