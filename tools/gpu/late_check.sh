#!/bin/bash
# attention kernel tests (incl. the non-fold fused-decode branch), then the profiled bench wave
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
timeout -k 10 300 python -u -m pytest tests/kernels/test_attention.py -x -q --timeout 120 --timeout-method thread > gpurun_out/attn_tests.log 2>&1 || { tail -30 gpurun_out/attn_tests.log; exit 1; }
tail -1 gpurun_out/attn_tests.log
bash tools/gpu/prof_r2g.sh
