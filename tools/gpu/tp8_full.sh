#!/bin/bash
# Full-depth Llama-3-70B TP=8 rehearsal on ONE MI355X: TP=1 reference (packed-only 70B), then 8
# ranks (each under rocprofv3 --kernel-trace), merged trace report; raw CSVs are deleted after.
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
cd $R
OUT=gpurun_out/tp8_full
timeout -k 10 1080 python -u tools/tp_rehearsal.py --world 8 --model llama3-70b --batch 64 --prompt 256 --steps 12 \
  --cmp-tokens 8 --ref ${REF:-run} --prof --timeout 1040 --out $OUT > gpurun_out/tp8_full.log 2>&1
rc=$?
echo "rehearsal rc=$rc"
tail -3 gpurun_out/tp8_full.log
if ls $OUT/trace_r0 >/dev/null 2>&1; then
  python tools/tp_gaps.py $OUT/trace_r0 $OUT/trace_r1 $OUT/trace_r2 $OUT/trace_r3 $OUT/trace_r4 $OUT/trace_r5 \
    $OUT/trace_r6 $OUT/trace_r7 --out $OUT/gaps.md > /dev/null 2>&1 || echo "gaps failed"
  find $OUT -name '*.csv' -delete
fi
exit $rc
