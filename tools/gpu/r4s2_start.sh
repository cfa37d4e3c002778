#!/bin/bash
# session-2: fused QKV -> attention tests (K/V prefetch variants), in-kernel stamps of the two
# fused decode launches, headline bench, PMC counters of the fused decode launches
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/kernels/test_attention.py \
  > gpurun_out/s2_attn_tests.log 2>&1 || { tail -40 gpurun_out/s2_attn_tests.log; exit 1; }
tail -2 gpurun_out/s2_attn_tests.log
timeout -k 10 150 python -u tools/qa_stamps.py > gpurun_out/s2_qa_stamps.txt 2>&1 || { tail -20 gpurun_out/s2_qa_stamps.txt; exit 1; }
cat gpurun_out/s2_qa_stamps.txt
timeout -k 10 120 python -u tools/mlp_stamps.py > gpurun_out/s2_mlp_stamps.txt 2>&1 || { tail -20 gpurun_out/s2_mlp_stamps.txt; exit 1; }
cat gpurun_out/s2_mlp_stamps.txt
timeout -k 10 400 python bench.py --steps 10 --warmup 2 > gpurun_out/s2_bench.json 2> gpurun_out/s2_bench.err || { tail -30 gpurun_out/s2_bench.err; exit 1; }
cat gpurun_out/s2_bench.json
bash $R/tools/gpu/fused_pmc.sh
