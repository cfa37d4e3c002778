#!/bin/bash
# round-4 end check on one MI355X after the prefill GEMM cleanup: GPU suite, smoke(), headline
# bench (10 waves), Mixtral bench (grouped prefill GEMM), 70B on one GPU (packed prefill GEMM)
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 700 python -u -m pytest -q --timeout 150 --timeout-method thread -m gpu tests \
  > gpurun_out/end_gpu_suite.log 2>&1; rc=$?
tail -8 gpurun_out/end_gpu_suite.log
[ $rc -eq 124 ] || [ $rc -eq 137 ] && exit 1
grep -q "Fatal Python error\|Segmentation fault\|core dumped" gpurun_out/end_gpu_suite.log && exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/end_smoke.log 2>&1 || { tail -20 gpurun_out/end_smoke.log; exit 1; }
tail -2 gpurun_out/end_smoke.log
timeout -k 10 400 python bench.py --steps 10 --warmup 2 > gpurun_out/end_bench.json 2> gpurun_out/end_bench.err || { tail -30 gpurun_out/end_bench.err; exit 1; }
cat gpurun_out/end_bench.json
timeout -k 10 400 python bench.py --model mixtral-8x7b --steps 2 > gpurun_out/end_mix.json 2> gpurun_out/end_mix.err || { tail -30 gpurun_out/end_mix.err; exit 1; }
cat gpurun_out/end_mix.json
timeout -k 10 500 python bench.py --model llama3-70b --steps 1 --warmup 1 > gpurun_out/end_70b.json 2> gpurun_out/end_70b.err || { tail -30 gpurun_out/end_70b.err; exit 1; }
cat gpurun_out/end_70b.json
