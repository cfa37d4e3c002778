#!/bin/bash
# TP decode collective driven by the GEMM epilogue (POLYKEY_TP_PUSH): correctness on one GPU
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=gpurun_out
P="python3 -u -m pytest -x -v --timeout 300 --timeout-method thread"
timeout -k 10 200 $P tests/kernels/test_gemm_skinny.py tests/kernels/test_phases.py -m gpu -q > $O/r5_push_kernels.log 2>&1 || { tail -30 $O/r5_push_kernels.log; exit 1; }
tail -1 $O/r5_push_kernels.log
timeout -k 10 400 $P tests/parallel/test_custom_ar_gpu.py > $O/r5_push_car.log 2>&1 || { tail -40 $O/r5_push_car.log; exit 1; }
tail -4 $O/r5_push_car.log
timeout -k 10 560 $P tests/parallel/test_tp8_shapes_gpu.py -k "pushed or on_one_gpu" > $O/r5_push_tp8.log 2>&1 || { tail -40 $O/r5_push_tp8.log; exit 1; }
tail -4 $O/r5_push_tp8.log
