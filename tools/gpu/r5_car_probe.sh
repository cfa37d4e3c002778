#!/bin/bash
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=gpurun_out
timeout -k 10 120 python3 tools/car_probe.py | tee -a $O/r5_car_probe.jsonl || exit 1
for v in car_norel car_noacq; do
  POLYKEY_LIB_LIBPK_COMM=$R/tools/lab/libpk_comm_$v.so timeout -k 10 120 python3 tools/car_probe.py | tee -a $O/r5_car_probe.jsonl || exit 1
done
