#!/bin/bash
# cooperative in-launch split-K SiLU reduction (every split reduces 1 / S of the rows): tests, A/B
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/kernels/test_phases.py \
  tests/parallel/test_tp_chain_gpu.py tests/kernels/test_gemm_skinny.py > $O/r5_coop_tests.log 2>&1; rc=$?; tail -2 $O/r5_coop_tests.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  for cfg in "0 0" "1 0" "0 1"; do
    set -- $cfg
    POLYKEY_GATE_UP_INLAUNCH=$1 POLYKEY_MLP_FUSED_SPLIT=$2 timeout -k 10 200 python3 tools/tp_solo.py --model llama3-70b --tp 8 --iters 30 \
      | cut -c1-120 | sed "s/^{/{\"gu_inlaunch\": $1, \"mlp_fused_split\": $2, /" | tee -a $O/r5_coop.jsonl || exit 1
  done
done
