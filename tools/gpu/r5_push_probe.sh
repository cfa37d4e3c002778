#!/bin/bash
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 200 python3 tools/push_probe.py | tee -a gpurun_out/r5_push_probe.jsonl || exit 1
for v in push_nofence push_nostore; do
  POLYKEY_LIB_LIBPK_KERNELS=$R/tools/lab/libpk_kernels_$v.so timeout -k 10 200 python3 tools/push_probe.py | tee -a gpurun_out/r5_push_probe.jsonl || exit 1
done
