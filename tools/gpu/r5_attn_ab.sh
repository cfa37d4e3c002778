#!/bin/bash
# 70B TP=8 decode attention: K/V prefetch across the q slab reduction (one workgroup per CU),
# write-through in-launch partition merge, 512-key partitions -- tests, per-rank step A/B, profile
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 240 --timeout-method thread \
  tests/kernels/test_phases.py -k "partition_merge" tests/kernels/test_attention.py tests/parallel/test_tp_chain_gpu.py \
  > $O/r5_attn_tests.log 2>&1; rc=$?; tail -3 $O/r5_attn_tests.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  for cfg in "1 0 256" "0 0 256" "1 1 256" "1 0 0" "0 0 0"; do
    set -- $cfg
    POLYKEY_DECODE_PRE=$1 POLYKEY_DECODE_INLAUNCH_MERGE=$2 POLYKEY_DECODE_FILL=$3 timeout -k 10 200 \
      python3 tools/tp_solo.py --model llama3-70b --tp 8 --iters 30 | cut -c1-130 | sed "s/^{/{\"pre\": $1, \"merge\": $2, \"fill\": $3, /" | tee -a $O/r5_attn_ab.jsonl || exit 1
  done
done
timeout -k 10 200 python3 tools/tp_solo.py --model llama3-8b --tp 1 --iters 30 | cut -c1-130 | tee -a $O/r5_attn_ab.jsonl || exit 1
cd /tmp && export TMPDIR=/tmp
POLYKEY_DECODE_INLAUNCH_MERGE=1 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d /tmp/s70 -- python3 $R/tools/tp_solo.py --model llama3-70b \
  --tp 8 --iters 10 --eager > /tmp/s70.log 2>&1 || { tail -20 /tmp/s70.log; exit 1; }
python3 $R/tools/kgrid.py /tmp/s70 $R/$O/r5_70b_attn_kgrid.md --per 13 > /dev/null
