#!/bin/bash
# 4-wave prefill GEMM load-path variants: numerics, then gate_up timing of each
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/kernels/test_gemm_prefill.py > gpurun_out/pg5_tests.log 2>&1 \
  || { tail -40 gpurun_out/pg5_tests.log; exit 1; }
tail -2 gpurun_out/pg5_tests.log
timeout -k 10 200 python -u tools/pg_probe.py ${PV:-4 5} > gpurun_out/pg5_probe.jsonl 2>&1 || { tail -20 gpurun_out/pg5_probe.jsonl; exit 1; }
grep '^{' gpurun_out/pg5_probe.jsonl
for v in ${ABL:-}; do
  POLYKEY_LIB_LIBPK_KERNELS=$PWD/tools/lab/libpk_kernels_$v.so timeout -k 10 120 python -u tools/pg_probe.py ${ABLV:-6} >> gpurun_out/pg5_probe.jsonl 2>&1 || { tail -20 gpurun_out/pg5_probe.jsonl; exit 1; }
done
grep '^{' gpurun_out/pg5_probe.jsonl | tail -2
