#!/bin/bash
# fused MLP gate_up tiles with a four-deep weight ring (production build) vs two-deep (lab build):
# bit-identity tests, then the graph-replayed 8B decode step alternating (tp_solo)
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=gpurun_out
timeout -k 10 300 python -u -m pytest tests/kernels/test_gemm_skinny.py -x -q --timeout 200 --timeout-method thread -k "mlp or fused" > $O/r6_wdeep_test.log 2>&1
rc=$?; tail -3 $O/r6_wdeep_test.log; [ $rc -eq 0 ] || exit $rc
rm -f $O/r6_wdeep.jsonl
for i in 1 2 3; do
  for v in deep w2; do
    if [ $v = w2 ]; then export POLYKEY_LIB_LIBPK_KERNELS=$R/tools/lab/libpk_kernels_mlp_w2.so; else unset POLYKEY_LIB_LIBPK_KERNELS; fi
    timeout -k 10 200 python3 tools/tp_solo.py --model llama3-8b --tp 1 --batch 64 --ctx 384 --iters 30 | cut -c1-140 \
      | sed "s/^{/{\"w\": \"$v\", /" | tee -a $O/r6_wdeep.jsonl || exit 1
  done
done
unset POLYKEY_LIB_LIBPK_KERNELS
