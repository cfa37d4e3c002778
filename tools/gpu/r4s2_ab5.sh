#!/bin/bash
# GPU suite (every failure listed), fused MLP down variants (NT / LDS prefetch / both), decode GEMMs at 256 / 512 rows
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 700 python -u -m pytest -q --timeout 150 --timeout-method thread -m gpu tests \
  > gpurun_out/ab5_gpu_suite.log 2>&1; rc=$?
tail -12 gpurun_out/ab5_gpu_suite.log
[ $rc -eq 124 ] || [ $rc -eq 137 ] && exit 1
grep -q "Fatal Python error\|Segmentation fault\|core dumped" gpurun_out/ab5_gpu_suite.log && exit 1
timeout -k 10 200 python -u tools/mlp_stamps.py > gpurun_out/ab5_mlp_stamps.txt 2>&1 || { tail -20 gpurun_out/ab5_mlp_stamps.txt; exit 1; }
head -3 gpurun_out/ab5_mlp_stamps.txt
timeout -k 10 300 python -u tools/wide_decode_probe.py > gpurun_out/ab5_wide.jsonl 2>&1 || { tail -20 gpurun_out/ab5_wide.jsonl; exit 1; }
cat gpurun_out/ab5_wide.jsonl
