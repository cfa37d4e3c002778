#!/bin/bash
# the TP collective carried by its consumer's launch (kernels/car_gemm.hip): correctness on the
# shared GPU (W = 4 / 8 ranks) and on loopback at 70B TP=8 shapes, then the per-rank step A/B
# (plain chain / carried, paired workgroups / carried, separate workgroups)
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=gpurun_out
TAG=${1:-b}
timeout -k 10 400 python -u -m pytest tests/parallel/test_custom_ar_gpu.py -x -v --timeout 300 --timeout-method thread > $O/r6_carry_test_$TAG.log 2>&1
rc=$?; tail -3 $O/r6_carry_test_$TAG.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  for v in "0 1" "1 1" "1 0"; do
    set -- $v
    POLYKEY_TP_CARRY=$1 POLYKEY_CAR_PAIRED=$2 timeout -k 10 200 python3 tools/tp_solo.py --model llama3-70b --tp 8 --iters 30 --car loopback \
      | cut -c1-300 | sed "s/^{/{\"carry\": $1, \"paired\": $2, /" | tee -a $O/r6_carry_ab_$TAG.jsonl || exit 1
  done
done
