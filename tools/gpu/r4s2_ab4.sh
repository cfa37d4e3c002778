#!/bin/bash
# full GPU suite (no -x: every failure listed), then the fused-launch A/Bs and the headline bench
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 700 python -u -m pytest -q --timeout 150 --timeout-method thread -m gpu tests \
  > gpurun_out/ab4_gpu_suite.log 2>&1; rc=$?
tail -25 gpurun_out/ab4_gpu_suite.log
[ $rc -eq 124 ] || [ $rc -eq 137 ] && exit 1
grep -q "Fatal Python error\|Segmentation fault\|core dumped" gpurun_out/ab4_gpu_suite.log && exit 1
timeout -k 10 200 python -u tools/qa_stamps.py > gpurun_out/ab4_qa_stamps.txt 2>&1 || { tail -20 gpurun_out/ab4_qa_stamps.txt; exit 1; }
head -3 gpurun_out/ab4_qa_stamps.txt
timeout -k 10 200 python -u tools/mlp_stamps.py > gpurun_out/ab4_mlp_stamps.txt 2>&1 || { tail -20 gpurun_out/ab4_mlp_stamps.txt; exit 1; }
head -3 gpurun_out/ab4_mlp_stamps.txt
timeout -k 10 400 python bench.py --steps 10 --warmup 2 > gpurun_out/ab4_bench.json 2> gpurun_out/ab4_bench.err || { tail -30 gpurun_out/ab4_bench.err; exit 1; }
cat gpurun_out/ab4_bench.json
