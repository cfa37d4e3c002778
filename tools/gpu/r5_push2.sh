#!/bin/bash
# push epilogue with write-through system-scope stores: correctness, then GEMM-side cost
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=gpurun_out
P="python3 -u -m pytest -x -v --timeout 300 --timeout-method thread"
timeout -k 10 400 $P tests/parallel/test_custom_ar_gpu.py > $O/r5_push2_car.log 2>&1 || { tail -40 $O/r5_push2_car.log; exit 1; }
tail -2 $O/r5_push2_car.log
timeout -k 10 300 $P tests/parallel/test_tp8_shapes_gpu.py -k pushed > $O/r5_push2_tp8.log 2>&1 || { tail -40 $O/r5_push2_tp8.log; exit 1; }
tail -2 $O/r5_push2_tp8.log
timeout -k 10 200 python3 tools/push_probe.py | tee $O/r5_push2_probe.jsonl
