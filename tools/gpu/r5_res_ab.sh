#!/bin/bash
# residual phase A/B: production (res phase off / on) vs the timing-only plain-load variant, then
# per-kernel stats of res off / on under rocprofv3
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=gpurun_out
for i in 1 2; do
  for v in off on plain; do
    lib=""; rp=1
    [ $v = off ] && rp=0
    [ $v = plain ] && lib=$R/tools/lab/libpk_kernels_res_plain.so
    POLYKEY_LIB_LIBPK_KERNELS=$lib POLYKEY_RES_PHASE=$rp POLYKEY_O_PHASE=0 timeout -k 10 200 python3 tools/tp_solo.py \
      --model llama3-8b --tp 1 --iters 30 | sed "s/^{/{\"v\": \"$v\", /" | tee -a $O/r5_res_ab.jsonl || exit 1
  done
done
cd /tmp && export TMPDIR=/tmp
for rp in 0 1; do
  POLYKEY_RES_PHASE=$rp POLYKEY_O_PHASE=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
    -d /tmp/res_$rp -- python3 $R/tools/tp_solo.py --model llama3-8b --tp 1 --iters 10 --eager > /tmp/res_$rp.log 2>&1 \
    || { tail -20 /tmp/res_$rp.log; exit 1; }
  python3 $R/tools/kstats.py /tmp/res_$rp $R/$O/r5_res${rp}_kstats.md 24 > /dev/null
done
python3 $R/tools/kgrid.py /tmp/res_0 $R/$O/r5_8b_kgrid.md --per 13 > /dev/null
SOLO=$R/tools/tp_solo.py
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d /tmp/s70 -- python3 $SOLO --model llama3-70b --tp 8 \
  --iters 10 --eager > /tmp/s70.log 2>&1 || { tail -20 /tmp/s70.log; exit 1; }
python3 $R/tools/kgrid.py /tmp/s70 $R/$O/r5_70b_kgrid.md --per 13 > /dev/null
