#!/bin/bash
# round-4 evidence pass: PMC counters of the fused decode kernels, the concurrency sweep,
# streaming / Mixtral / 70B-on-one-GPU benches
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
bash $R/tools/gpu/fused_pmc.sh || exit 1
cd $R
rm -f gpurun_out/conc_sweep.jsonl
CONC="64 128 256 512" STEPS=2 bash tools/gpu/conc_sweep.sh || exit 1
timeout -k 10 300 python bench.py --steps 5 --mode stream > gpurun_out/fb_stream.json 2> gpurun_out/fb_stream.err || exit 1
cat gpurun_out/fb_stream.json
timeout -k 10 400 python bench.py --model mixtral-8x7b --steps 2 > gpurun_out/fb_mix.json 2> gpurun_out/fb_mix.err || exit 1
cat gpurun_out/fb_mix.json
