#!/bin/bash
# prefill GEMM load placement: A / W of the next tile split over the two sub-steps (lab build), correctness then A/B
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=gpurun_out
POLYKEY_LIB_LIBPK_KERNELS=$R/tools/lab/libpk_kernels_pb_split.so timeout -k 10 300 python -u -m pytest tests/kernels/test_gemm_prefill.py -x -q --timeout 120 --timeout-method thread > $O/r6_psplit_test.log 2>&1
rc=$?; tail -3 $O/r6_psplit_test.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 tools/prefill_gemm_ab.py 4 6 | tee $O/r6_psplit.txt || exit 1
for v in pb_split pb_novm; do
  echo "== $v" | tee -a $O/r6_psplit.txt
  POLYKEY_LIB_LIBPK_KERNELS=$R/tools/lab/libpk_kernels_$v.so timeout -k 10 300 python3 tools/prefill_gemm_ab.py 4 6 | tee -a $O/r6_psplit.txt || exit 1
done
