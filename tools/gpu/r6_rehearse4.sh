#!/bin/bash
# the driver's N = 4 children rehearsed with 4 ranks sharing one MI355X: Llama-3-70B TP = 4 (full
# depth: serving preflight, graphs vs eager tokens, timed decode) and Mixtral-8x7B DP attention +
# EP = 4 through bench.py (IPC expert all-to-all among 4 processes)
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=gpurun_out
timeout -k 10 600 python3 tools/tp_rehearsal.py --world 4 --model llama3-70b --batch 16 --prompt 64 --steps 8 \
  --cmp-tokens 4 --ref none --timeout 500 --hw-queues 1 --out $R/gpurun_out/rh4 > $O/r6_rehearse_tp4.log 2>&1 \
  || { tail -30 $O/r6_rehearse_tp4.log; tail -30 $R/gpurun_out/rh4/rank0.log; exit 1; }
tail -4 $O/r6_rehearse_tp4.log
[ -n "$TP_ONLY" ] && exit 0
GPU_MAX_HW_QUEUES=1 timeout -k 10 500 python -u bench.py --gpus 4 --tp 1 --ep 4 --model mixtral-8x7b --steps 1 \
  --warmup 1 --num-kv-blocks 1024 --tp-extra-model none --ep-extra-model none > $O/r6_rehearse_ep4.log 2>&1 \
  || { tail -30 $O/r6_rehearse_ep4.log; exit 1; }
grep '^{"metric"' $O/r6_rehearse_ep4.log | cut -c1-600
