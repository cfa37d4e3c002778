#!/bin/bash
# ablations of the buffer-load prefill GEMM (variant 8; timing only): no vmcnt wait / no loads in the k-loop
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=gpurun_out
for v in pb_novm pb_noload; do
  echo "== $v" | tee -a $O/r6_pbuf_ablate.txt
  POLYKEY_LIB_LIBPK_KERNELS=$R/tools/lab/libpk_kernels_$v.so timeout -k 10 300 python3 tools/prefill_gemm_ab.py 6 8 | tee -a $O/r6_pbuf_ablate.txt || exit 1
done
