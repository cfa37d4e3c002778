#!/bin/bash
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 240 --timeout-method thread \
  tests/kernels/test_phases.py tests/kernels/test_attention.py tests/parallel/test_tp_chain_gpu.py tests/e2e/test_engine_gpu.py \
  > $O/r5_attn_tests.log 2>&1; rc=$?; tail -3 $O/r5_attn_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 tools/attn70_probe.py | cut -c1-100 | tee $O/r5_attn70_probe2.jsonl || exit 1
timeout -k 10 300 python3 tools/attn70_probe.py --heads 32,8 | cut -c1-100 | tee $O/r5_attn8b_probe2.jsonl || exit 1
for cfg in "1 256" "0 256" "0 0" "1 0"; do
  set -- $cfg
  POLYKEY_DECODE_PRE=$1 POLYKEY_DECODE_FILL=$2 timeout -k 10 200 python3 tools/tp_solo.py --model llama3-70b --tp 8 --iters 30 \
    | cut -c1-130 | sed "s/^{/{\"pre\": $1, \"fill\": $2, /" | tee -a $O/r5_attn_ab4.jsonl || exit 1
done
timeout -k 10 200 python3 tools/tp_solo.py --model llama3-8b --tp 1 --iters 30 | cut -c1-130 | tee -a $O/r5_attn_ab4.jsonl || exit 1
POLYKEY_QKV_ATTN_FUSED=0 timeout -k 10 200 python3 tools/tp_solo.py --model llama3-8b --tp 1 --iters 30 | cut -c1-130 | sed "s/^{/{\"unfused\": 1, /" | tee -a $O/r5_attn_ab4.jsonl || exit 1
