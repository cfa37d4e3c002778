#!/bin/bash
# fused decode launches: K/V prefetch depth x QKV n-block height, non-temporal down weights (A/B
# with stamps), tests of every variant, PMC counters of the fused kernels
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/kernels/test_attention.py tests/kernels/test_gemm_skinny.py \
  > gpurun_out/ab1_attn_tests.log 2>&1 || { tail -40 gpurun_out/ab1_attn_tests.log; exit 1; }
tail -1 gpurun_out/ab1_attn_tests.log
timeout -k 10 200 python -u tools/qa_stamps.py > gpurun_out/ab1_qa_stamps.txt 2>&1 || { tail -20 gpurun_out/ab1_qa_stamps.txt; exit 1; }
cat gpurun_out/ab1_qa_stamps.txt
timeout -k 10 150 python -u tools/mlp_stamps.py > gpurun_out/ab1_mlp_stamps.txt 2>&1 || { tail -20 gpurun_out/ab1_mlp_stamps.txt; exit 1; }
cat gpurun_out/ab1_mlp_stamps.txt
bash $R/tools/gpu/r4s2_ab2.sh
bash $R/tools/gpu/fused_pmc.sh
