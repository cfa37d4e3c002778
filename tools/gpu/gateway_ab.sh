#!/bin/bash
# A/B of the DP front ends with 4 ranks sharing one MI355X (Llama-3-8B, 64 clients per rank):
# per-rank endpoints vs the SO_REUSEPORT gateway (one address, an acceptor per rank).
R=$GRAFT_REPO_ROOT
cd $R
for fe in replicas gateway replicas gateway; do
  POLYKEY_BENCH_TIMING=1 GPU_MAX_HW_QUEUES=1 timeout -k 10 420 python -u bench.py --gpus 4 --steps 2 --warmup 1 --num-kv-blocks 1300 \
    --frontend $fe > gpurun_out/gw_$fe.log 2>&1 || { echo "bench $fe failed"; tail -20 gpurun_out/gw_$fe.log; exit 1; }
  grep '^{"metric"' gpurun_out/gw_$fe.log | tee -a gpurun_out/gateway_ab.jsonl
done
