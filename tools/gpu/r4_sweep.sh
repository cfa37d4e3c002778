#!/bin/bash
# concurrency sweep 128 / 256 / 512 on HEAD, then the 8B decode-step variant A/Bs
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
rm -f gpurun_out/conc_sweep.jsonl
CONC="128 256 512" STEPS=1 bash tools/gpu/conc_sweep.sh || exit 1
sed -i 's/for i in 1 2; do/for i in 1; do/' tools/gpu/r4s2_ab9.sh
sed -i '$d' tools/gpu/r4s2_ab9.sh
bash tools/gpu/r4s2_ab9.sh
