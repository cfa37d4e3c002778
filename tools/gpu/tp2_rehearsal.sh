#!/bin/bash
# TP=2 rehearsal (8B, both ranks on one GPU), each rank under its own kernel trace; merged gaps
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
export MASTER_ADDR=127.0.0.1 MASTER_PORT=29555
timeout -k 10 420 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/tp2_r0 -- python3 $R/tools/tp2_rehearsal.py --rank 0 --out $R/gpurun_out/tp2.json > $R/gpurun_out/tp2_r0.log 2>&1 &
p0=$!
timeout -k 10 420 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/tp2_r1 -- python3 $R/tools/tp2_rehearsal.py --rank 1 > $R/gpurun_out/tp2_r1.log 2>&1 &
p1=$!
wait $p0; rc0=$?
wait $p1; rc1=$?
echo "rc0=$rc0 rc1=$rc1"
tail -3 $R/gpurun_out/tp2_r0.log $R/gpurun_out/tp2_r1.log
[ $rc0 -eq 0 ] && [ $rc1 -eq 0 ] || exit 1
cd $R
python3 tools/tp2_gaps.py gpurun_out/tp2_r0 gpurun_out/tp2_r1 gpurun_out/tp2_gaps.md || exit 1
find gpurun_out/tp2_r0 gpurun_out/tp2_r1 -name '*kernel_trace.csv' -delete
exit 0
