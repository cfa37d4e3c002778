#!/bin/bash
# Decode above 64 rows: row-tile kernel tests, GEMM micro-bench vs hipBLASLt, concurrency sweep.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/kernels/test_gemm_skinny.py \
  tests/parallel/test_tp_rank_death_gpu.py > gpurun_out/rows_tests.log 2>&1 || { tail -40 gpurun_out/rows_tests.log; exit 1; }
tail -3 gpurun_out/rows_tests.log
timeout -k 10 300 python -u tools/bench_gemm_rows.py > gpurun_out/rows_gemm.jsonl 2> gpurun_out/rows_gemm.err \
  || { tail -20 gpurun_out/rows_gemm.err; exit 1; }
cat gpurun_out/rows_gemm.jsonl
CONC="${CONC:-64 128 256 512}" bash tools/gpu/conc_sweep.sh
