#!/bin/bash
# headline bench: prefill token budget 8192 (default) vs 16384 (one prefill step per wave), alternating
set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/ab_budget.txt
for b in 8192 16384 8192 16384; do
  timeout -k 10 300 python bench.py --steps 4 --max-batched-tokens $b > gpurun_out/b_$b.json 2> gpurun_out/b_$b.err || exit 1
  python -c "import json,sys; d=json.load(open('gpurun_out/b_$b.json')); print($b, d['value'], d['ms_per_step'], d['p50_e2e_latency_ms'])" >> gpurun_out/ab_budget.txt
done
