#!/bin/bash
# 4-wave prefill GEMM (variants 6 / 7): numerics, then A/B against the 8-wave deep kernel and hipBLASLt
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/kernels/test_gemm_prefill.py > gpurun_out/pg4_tests.log 2>&1 \
  || { tail -40 gpurun_out/pg4_tests.log; exit 1; }
tail -3 gpurun_out/pg4_tests.log
timeout -k 10 300 python -u tools/prefill_gemm_ab.py ${VA:-4} ${VB:-4} > gpurun_out/pg4_ab.jsonl 2>&1 || { tail -20 gpurun_out/pg4_ab.jsonl; exit 1; }
cat gpurun_out/pg4_ab.jsonl
