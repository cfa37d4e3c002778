#!/bin/bash
# 8B at 256 concurrent clients: gate_up on hipBLASLt (+ norm / SiLU kernels) above 192 vs 384 rows,
# alternating; then the 128 / 512 points of the sweep on HEAD
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
rm -f gpurun_out/ab8.jsonl
for i in 1 2; do
  for t in 384 192; do
    POLYKEY_AB_GATE_UP_MAX_M=$t timeout -k 10 400 python -u bench.py --steps 1 --warmup 1 --concurrency 256 \
      > gpurun_out/ab8_$t.log 2>&1 || { tail -30 gpurun_out/ab8_$t.log; exit 1; }
    echo "{\"gate_up_max_m\": $t, \"line\": $(grep '^{"metric"' gpurun_out/ab8_$t.log)}" | tee -a gpurun_out/ab8.jsonl
  done
done
