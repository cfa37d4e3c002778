#!/bin/bash
# fused MLP variants (non-temporal down weights, LDS prefetch of down k-steps): tests, interleaved timing;
# then the headline bench on the K/V-prefetch fused attention and the PMC passes
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/kernels/test_attention.py \
  tests/kernels/test_gemm_skinny.py > gpurun_out/ab3_tests.log 2>&1 || { tail -40 gpurun_out/ab3_tests.log; exit 1; }
tail -1 gpurun_out/ab3_tests.log
timeout -k 10 200 python -u tools/qa_stamps.py > gpurun_out/ab3_qa_stamps.txt 2>&1 || { tail -20 gpurun_out/ab3_qa_stamps.txt; exit 1; }
cat gpurun_out/ab3_qa_stamps.txt
timeout -k 10 200 python -u tools/mlp_stamps.py > gpurun_out/ab3_mlp_stamps.txt 2>&1 || { tail -20 gpurun_out/ab3_mlp_stamps.txt; exit 1; }
cat gpurun_out/ab3_mlp_stamps.txt
timeout -k 10 400 python bench.py --steps 10 --warmup 2 > gpurun_out/ab3_bench.json 2> gpurun_out/ab3_bench.err || { tail -30 gpurun_out/ab3_bench.err; exit 1; }
cat gpurun_out/ab3_bench.json
bash $R/tools/gpu/fused_pmc.sh 2>&1 | tail -30
