#!/bin/bash
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=gpurun_out
P="python3 -u -m pytest -x -v --timeout 300 --timeout-method thread"
timeout -k 10 300 $P tests/parallel/test_custom_ar_gpu.py > $O/r5_carpre_car.log 2>&1 || { tail -40 $O/r5_carpre_car.log; exit 1; }
tail -2 $O/r5_carpre_car.log
timeout -k 10 120 python3 tools/car_probe.py | tee -a $O/r5_car_probe.jsonl || exit 1
for i in 1 2; do
  timeout -k 10 200 python3 tools/tp_solo.py --model llama3-70b --tp 8 --iters 30 --car loopback | cut -c1-150 \
      | sed "s/^{/{\"car_pre\": 1, /" | tee -a $O/r5_loopback.jsonl || exit 1
done
