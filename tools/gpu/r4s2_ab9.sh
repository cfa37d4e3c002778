#!/bin/bash
# 8B graph-captured decode step A/Bs (tools/tp_solo.py), alternating on one box: production vs
# hand-off pollers sleeping 4 (variant build), QKV split 2 in the fused launch, o-projection split 8
# (64-row tiles) / 128-row tiles at split 8
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
rm -f gpurun_out/ab9.jsonl
run() {  # tag, env...
  local tag=$1; shift
  env "$@" timeout -k 10 300 python -u tools/tp_solo.py --model llama3-8b --tp 1 --iters 30 > gpurun_out/ab9_$tag.log 2>&1 \
    || { tail -20 gpurun_out/ab9_$tag.log; return 1; }
  echo "{\"variant\": \"$tag\", \"line\": $(tail -1 gpurun_out/ab9_$tag.log)}" | tee -a gpurun_out/ab9.jsonl
}
for i in 1 2; do
  run prod POLYKEY_AB_X=0 || exit 1
  run sleep4 POLYKEY_LIB_LIBPK_KERNELS=$R/tools/lab/libpk_kernels_sleep4.so || exit 1
  run qkvS2 POLYKEY_AB_QKV_S=2 || exit 1
  run oS8 POLYKEY_AB_O_S=8 || exit 1
  run oFull POLYKEY_AB_O_HALF=0 || exit 1
done
bash $R/tools/gpu/r4s2_ab10.sh
