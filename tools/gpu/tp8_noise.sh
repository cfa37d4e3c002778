#!/bin/bash
# Noise calibration for the 70B TP=8 vs TP=1 logits comparison (tools/tp_rehearsal.py --role noise)
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 900 python -u tools/tp_rehearsal.py --role noise --model llama3-70b --max-batched 8192 \
  --out gpurun_out/tp8_noise > gpurun_out/tp8_noise.log 2>&1
rc=$?
tail -2 gpurun_out/tp8_noise.log
exit $rc
