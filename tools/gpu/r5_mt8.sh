#!/bin/bash
# 128-row decode tiles staging A per 256-deep chunk (variant build) vs per 128-deep step
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=gpurun_out
V=$R/tools/lab/libpk_kernels_mt8_chunk256.so
POLYKEY_LIB_LIBPK_KERNELS=$V timeout -k 10 400 python -u -m pytest --deselect "tests/kernels/test_gemm_skinny.py::test_mlp_fused_matches_two_launches" -x -q --timeout 240 --timeout-method thread \
  tests/kernels/test_gemm_skinny.py tests/e2e/test_engine_gpu.py -k "large_decode or skinny or rows" > $O/r5_mt8_tests.log 2>&1; rc=$?; tail -2 $O/r5_mt8_tests.log; true
for i in 1 2; do
  for v in base mt8; do
    if [ $v = mt8 ]; then export POLYKEY_LIB_LIBPK_KERNELS=$V; else unset POLYKEY_LIB_LIBPK_KERNELS; fi
    for b in 128 256; do
      timeout -k 10 200 python3 tools/tp_solo.py --model llama3-8b --tp 1 --batch $b --iters 20 | cut -c1-110 | sed "s/^{/{\"lib\": \"$v\", /" | tee -a $O/r5_mt8.jsonl || exit 1
    done
  done
done
