#!/bin/bash
# P7 prefill half: 2 ranks (IPC collectives) on one GPU, 8B shapes, 4 layers, 4 x 1000-token prompts
# in one 4000-row prefill step -> 4 row chunks of 1000 (8 MB each: inside the custom all-reduce's
# 16 MB slot; 2000-row chunks fell back to gloo in round 5); each rank under a kernel trace, then
# the comm-stream kernels' overlap with the compute stream per rank.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=gpurun_out
rm -rf /tmp/ov
POLYKEY_SEQUENCE_PARALLEL=0 timeout -k 10 400 python3 tools/tp_rehearsal.py --world 2 --model llama3-8b --layers 4 --batch 4 --prompt 1000 --steps 4 \
  --cmp-tokens 2 --max-batched 8192 --ref none --prof --timeout 300 --hw-queues 0 --out /tmp/ov > $O/r6_ov.log 2>&1 \
  || { tail -20 $O/r6_ov.log; tail -30 /tmp/ov/rank0.log; exit 1; }
tail -2 $O/r6_ov.log
for r in 0 1; do python3 tools/overlap_report.py /tmp/ov/trace_r$r $O/r6_overlap_r$r.md > /dev/null || exit 1; done
head -30 $O/r6_overlap_r0.md
timeout -k 10 120 python3 tools/lm_head_probe.py 64 | tee $O/r6_lm_head_probe.jsonl
