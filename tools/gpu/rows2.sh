#!/bin/bash
# row-tile split target / gate_up-on-hipBLASLt check: GEMM + e2e tests, then the concurrency sweep
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/kernels/test_gemm_skinny.py \
  tests/e2e/test_engine_gpu.py tests/e2e/test_real_width_gpu.py > gpurun_out/rows2_tests.log 2>&1 \
  || { tail -40 gpurun_out/rows2_tests.log; exit 1; }
tail -2 gpurun_out/rows2_tests.log
rm -f gpurun_out/conc_sweep.jsonl
CONC="${CONC:-64 256 512}" bash tools/gpu/conc_sweep.sh
