#!/bin/bash
# two 8B replicas sharing ONE MI355X (gloo control plane): one gRPC endpoint per rank (replicas)
# vs one front end on rank 0 routing to both engine processes (gateway); alternating
set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/ab_gateway.txt
for fe in replicas gateway replicas gateway; do
  timeout -k 10 400 python bench.py --gpus 2 --steps 3 --warmup 1 --gpu-mem-fraction 0.4 --frontend $fe \
    > gpurun_out/gw_$fe.json 2> gpurun_out/gw_$fe.err || exit 1
  python -c "import json; d=json.loads(open('gpurun_out/gw_$fe.json').read().strip().splitlines()[-1]); print('$fe', d['value'], d['ms_per_step'], d['p50_e2e_latency_ms'], d['config']['parallelism'])" >> gpurun_out/ab_gateway.txt
done
