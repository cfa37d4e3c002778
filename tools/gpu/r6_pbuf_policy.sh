#!/bin/bash
# cache-policy variants of the prefill GEMM's staging loads (lab builds), variant 6 in each vs hipBLASLt
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=gpurun_out
timeout -k 10 300 python3 tools/prefill_gemm_ab.py 4 6 | tee -a $O/r6_pbuf_policy.txt || exit 1
for v in pb_sc0_w pb_sc0_a pb_nt_w; do
  echo "== $v" | tee -a $O/r6_pbuf_policy.txt
  POLYKEY_LIB_LIBPK_KERNELS=$R/tools/lab/libpk_kernels_$v.so timeout -k 10 300 python3 tools/prefill_gemm_ab.py 4 6 | tee -a $O/r6_pbuf_policy.txt || exit 1
done
