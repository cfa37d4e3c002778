#!/bin/bash
# collectives with system-scope slot accesses and no fences: correctness, then timing
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=gpurun_out
P="python3 -u -m pytest -x -v --timeout 300 --timeout-method thread"
timeout -k 10 300 $P tests/parallel/test_custom_ar_gpu.py > $O/r5_carsys_car.log 2>&1 || { tail -40 $O/r5_carsys_car.log; exit 1; }
tail -2 $O/r5_carsys_car.log
timeout -k 10 900 $P tests/parallel/test_tp8_shapes_gpu.py > $O/r5_carsys_tp8.log 2>&1 || { tail -40 $O/r5_carsys_tp8.log; exit 1; }
tail -2 $O/r5_carsys_tp8.log
timeout -k 10 120 python3 tools/car_probe.py | tee -a $O/r5_car_probe.jsonl || exit 1
for i in 1 2; do
  for v in 0 1; do
    POLYKEY_TP_PUSH=$v timeout -k 10 200 python3 tools/tp_solo.py --model llama3-70b --tp 8 --iters 30 --car loopback | cut -c1-150 \
      | sed "s/^{/{\"push\": $v, \"car_sys\": 1, /" | tee -a $O/r5_loopback.jsonl || exit 1
  done
done
