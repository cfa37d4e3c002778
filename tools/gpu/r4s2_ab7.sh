#!/bin/bash
# whole-slice O tiles: tests; then the 8B graph-captured decode step (tools/tp_solo.py) of the
# production build vs variant builds of the same sources (tools/lab/build_variant.py), alternating
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 500 python -u -m pytest -x -q --timeout 150 --timeout-method thread -m gpu tests/kernels/test_gemm_skinny.py \
  tests/kernels/test_attention.py tests/e2e/test_real_width_gpu.py > gpurun_out/ab7_tests.log 2>&1 || { tail -40 gpurun_out/ab7_tests.log; exit 1; }
tail -1 gpurun_out/ab7_tests.log
rm -f gpurun_out/ab7_solo.jsonl
for i in 1 2 3; do
  for v in ${VARIANTS:-prod pre0 mlp_nt}; do
    if [ $v = prod ]; then lib=""; else lib=$R/tools/lab/libpk_kernels_$v.so; fi
    POLYKEY_LIB_LIBPK_KERNELS=$lib timeout -k 10 300 python -u tools/tp_solo.py --model llama3-8b --tp 1 --iters 30 \
      > gpurun_out/ab7_$v.log 2>&1 || { tail -20 gpurun_out/ab7_$v.log; exit 1; }
    echo "{\"variant\": \"$v\", \"line\": $(tail -1 gpurun_out/ab7_$v.log)}" | tee -a gpurun_out/ab7_solo.jsonl
  done
done
