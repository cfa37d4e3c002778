#!/bin/bash
# DP front-end A/B (4 ranks on one GPU) then the Mixtral EP=2 vs EP=1 rehearsal (2 ranks on one GPU)
cd $GRAFT_REPO_ROOT
bash tools/gpu/gateway_ab.sh && bash tools/gpu/ep_bench.sh
