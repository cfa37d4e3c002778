#!/bin/bash
# the prefill GEMM without its XOR chunk swizzle (lab build): correctness, A/B, stride probe
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=gpurun_out
L=$R/tools/lab/libpk_kernels_pb_noswz.so
POLYKEY_LIB_LIBPK_KERNELS=$L timeout -k 10 300 python -u -m pytest tests/kernels/test_gemm_prefill.py -x -q --timeout 120 --timeout-method thread > $O/r6_noswz_test.log 2>&1
rc=$?; tail -3 $O/r6_noswz_test.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 tools/prefill_gemm_ab.py 4 6 | tee $O/r6_noswz_ab.txt || exit 1
echo "== noswz" | tee -a $O/r6_noswz_ab.txt
POLYKEY_LIB_LIBPK_KERNELS=$L timeout -k 10 300 python3 tools/prefill_gemm_ab.py 4 6 | tee -a $O/r6_noswz_ab.txt || exit 1
timeout -k 10 300 python3 tools/prefill_stride_probe.py | tee $O/r6_stride_probe.jsonl
