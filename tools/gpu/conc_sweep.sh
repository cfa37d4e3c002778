#!/bin/bash
# Concurrency sweep of the 8B headline config on one MI355X: 64 / 128 / 256 / 512 concurrent
# unary gRPC clients (prompt 256, output 256), one JSON line each -> gpurun_out/conc_sweep.jsonl
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for c in ${CONC:-64 128 256 512}; do
  timeout -k 10 400 python -u bench.py --steps ${STEPS:-1} --warmup 1 --concurrency $c > gpurun_out/conc_$c.log 2>&1 \
    || { echo "bench c=$c failed"; tail -30 gpurun_out/conc_$c.log; exit 1; }
  grep '^{"metric"' gpurun_out/conc_$c.log | tee -a gpurun_out/conc_sweep.jsonl
done
