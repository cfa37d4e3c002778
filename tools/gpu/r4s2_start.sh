#!/bin/bash
# session-2 start: headline bench on HEAD, PMC counters of the fused decode launches
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 400 python bench.py --steps 10 --warmup 2 > gpurun_out/s2_bench.json 2> gpurun_out/s2_bench.err || { tail -30 gpurun_out/s2_bench.err; exit 1; }
cat gpurun_out/s2_bench.json
bash $R/tools/gpu/fused_pmc.sh
