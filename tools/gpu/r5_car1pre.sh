#!/bin/bash
# one-shot fused collective with the slab prefetch: W = 2 / 4 / 8 bit identity, then the 70B TP=2 rank
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=gpurun_out
timeout -k 10 300 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests/parallel/test_custom_ar_gpu.py > $O/r5_car1pre.log 2>&1 || { tail -40 $O/r5_car1pre.log; exit 1; }
tail -2 $O/r5_car1pre.log
for i in 1 2; do
  timeout -k 10 300 python3 tools/tp_solo.py --model llama3-70b --tp 2 --iters 20 --car loopback | cut -c1-160 | sed "s/^{/{\"car1_pre\": 1, /" | tee -a $O/r5_tp24_loop.jsonl || exit 1
done
