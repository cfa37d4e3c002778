#!/bin/bash
# concurrency sweep 64 / 128 / 256 / 512 on HEAD
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
rm -f gpurun_out/conc_sweep.jsonl
CONC="64 128 256 512" STEPS=2 bash tools/gpu/conc_sweep.sh || exit 1
