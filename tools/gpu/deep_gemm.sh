#!/bin/bash
# prefill GEMM numerics (incl. the deep-pipelined variants 4 / 5 and their bitwise race screen),
# then the shape bench
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/kernels/test_gemm_prefill.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t_pg.log 2>&1 && \
timeout -k 10 300 python tools/prefill_gemm_bench.py > gpurun_out/prefill_gemm.txt 2>&1
