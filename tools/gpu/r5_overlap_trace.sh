#!/bin/bash
# prefill TP overlap evidence: 2 ranks (IPC collectives) on one GPU, 8B shapes, 4 layers, 8 x 256-token
# prompts in one 2048-token prefill step (4 row chunks of 512); each rank under a kernel trace.
# Sequence parallelism off: its reduce-scatter / all-gather go through gloo between two ranks of
# one GPU (host-synchronous), the all-reduce of tp_row_parallel_overlapped through the IPC kernels
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=gpurun_out
rm -rf /tmp/ov
POLYKEY_SEQUENCE_PARALLEL=0 timeout -k 10 400 python3 tools/tp_rehearsal.py --world 2 --model llama3-8b --layers 4 --batch 8 --prompt 1000 --steps 4 \
  --cmp-tokens 2 --max-batched 8192 --ref none --prof --timeout 300 --out /tmp/ov > $O/r5_ov.log 2>&1 \
  || { tail -20 $O/r5_ov.log; tail -30 /tmp/ov/rank0.log; exit 1; }
tail -2 $O/r5_ov.log
for r in 0 1; do python3 tools/overlap_report.py /tmp/ov/trace_r$r $O/r5_overlap_r$r.md > /dev/null || exit 1; done
