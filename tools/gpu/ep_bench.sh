#!/bin/bash
# Mixtral-8x7B DP-attention + EP=2 (IPC expert all-to-all, graph-captured decode) vs two DP
# replicas (EP=1), both as 2 ranks sharing ONE MI355X -> gpurun_out/ep_bench.jsonl
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for ep in 2 1; do
  GPU_MAX_HW_QUEUES=1 timeout -k 10 500 python -u bench.py --gpus 2 --tp 1 --ep $ep --model mixtral-8x7b --steps ${STEPS:-2} \
    --warmup 1 --num-kv-blocks 2048 > gpurun_out/ep_bench_$ep.log 2>&1 \
    || { echo "ep=$ep failed"; tail -30 gpurun_out/ep_bench_$ep.log; exit 1; }
  grep '^{"metric"' gpurun_out/ep_bench_$ep.log | tee -a gpurun_out/ep_bench.jsonl
done
