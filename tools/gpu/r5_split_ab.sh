#!/bin/bash
# decode GEMM split A/B (QKV split, workgroup target of choose_split) on the per-rank step
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=gpurun_out
for cfg in "0 192" "16 192" "4 192" "0 256" "0 384" "0 192"; do
  set -- $cfg
  POLYKEY_QKV_SPLIT=$1 POLYKEY_SKINNY_TARGET=$2 timeout -k 10 200 python3 tools/tp_solo.py --model llama3-70b --tp 8 --iters 30 \
    | cut -c1-130 | sed "s/^{/{\"qkv_split\": $1, \"target\": $2, /" | tee -a $O/r5_split_ab.jsonl || exit 1
done
for t in 192 256 384; do
  POLYKEY_SKINNY_TARGET=$t timeout -k 10 200 python3 tools/tp_solo.py --model llama3-8b --tp 1 --iters 30 \
    | cut -c1-130 | sed "s/^{/{\"target\": $t, /" | tee -a $O/r5_split_ab.jsonl || exit 1
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d /tmp/s70 -- python3 $R/tools/tp_solo.py --model llama3-70b \
  --tp 8 --iters 10 --eager > /tmp/s70.log 2>&1 || { tail -20 /tmp/s70.log; exit 1; }
python3 $R/tools/kgrid.py /tmp/s70 $R/$O/r5_70b_kgrid_b.md --per 13 > /dev/null
