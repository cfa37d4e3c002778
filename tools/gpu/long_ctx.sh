#!/bin/bash
# graph-captured 8B decode step at 1k / 4k / ~8k context, 64 sequences (round-2 code)
set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/long_ctx.txt
for p in 1024 4096 7936; do
  timeout -k 10 400 python tools/ab_decode.py --prompt $p --steps 64 --reps 2 --tag ctx$p >> gpurun_out/long_ctx.txt 2> gpurun_out/long_ctx.err || exit 1
done
