#!/bin/bash
# 70B TP=8 shard, per-rank graph-captured decode step (tools/tp_solo.py), alternating: the decode
# attention fed by the QKV slabs (prod) vs QKV slabs reduced once by the RoPE / cache kernel then
# attention on q (red), + the partitions merged in-launch (red_inl)
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
rm -f gpurun_out/ab10.jsonl
run() {  # tag, env...
  local tag=$1; shift
  env "$@" timeout -k 10 400 python -u tools/tp_solo.py --model llama3-70b --tp 8 --iters 20 > gpurun_out/ab10_$tag.log 2>&1 \
    || { tail -20 gpurun_out/ab10_$tag.log; return 1; }
  echo "{\"variant\": \"$tag\", \"line\": $(tail -1 gpurun_out/ab10_$tag.log)}" | tee -a gpurun_out/ab10.jsonl
}
for i in ${REPS:-1}; do
  run prod POLYKEY_AB_X=0 || exit 1
  run red POLYKEY_AB_TP_REDUCE=1 || exit 1
  run red_inl POLYKEY_AB_TP_REDUCE=1 POLYKEY_AB_DECODE_MERGE_INLAUNCH=1 || exit 1
  run qkvh POLYKEY_AB_QKV_HALF=1 || exit 1
  run guh POLYKEY_AB_GU_HALF=1 || exit 1
  run red_qkvh POLYKEY_AB_TP_REDUCE=1 POLYKEY_AB_QKV_HALF=1 || exit 1
done
