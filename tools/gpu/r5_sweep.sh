#!/bin/bash
# round-5 evidence: 8B concurrency sweep (2 waves each), Mixtral and 70B-on-one-GPU benches
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out
rm -f gpurun_out/conc_sweep.jsonl
CONC="128 256 512" STEPS=2 bash tools/gpu/conc_sweep.sh || exit 1
cp gpurun_out/conc_sweep.jsonl gpurun_out/r5_conc_sweep.jsonl
timeout -k 10 400 python bench.py --model mixtral-8x7b --steps 2 > gpurun_out/r5_mix.json 2> gpurun_out/r5_mix.err || { tail -20 gpurun_out/r5_mix.err; exit 1; }
cat gpurun_out/r5_mix.json
timeout -k 10 500 python bench.py --model llama3-70b --steps 1 --warmup 1 > gpurun_out/r5_70b_tp1.json 2> gpurun_out/r5_70b_tp1.err || { tail -20 gpurun_out/r5_70b_tp1.err; exit 1; }
cat gpurun_out/r5_70b_tp1.json
