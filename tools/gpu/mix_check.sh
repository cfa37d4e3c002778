#!/bin/bash
# MoE / decode GEMM / engine GPU tests, then the Mixtral bench and a kernel trace of one wave
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R && timeout -k 10 400 python -u -m pytest tests/kernels/test_moe.py tests/kernels/test_gemm_skinny.py tests/e2e/test_engine_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t_mix.log 2>&1 && \
timeout -k 10 400 python bench.py --model mixtral-8x7b --steps 2 --warmup 1 > gpurun_out/bench_mix.json 2> gpurun_out/bench_mix.err && \
cd /tmp && export TMPDIR=/tmp && \
timeout -k 10 500 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/prof_mix3 -- python3 $R/bench.py --model mixtral-8x7b --steps 1 --warmup 1 > $R/gpurun_out/prof_mix3.log 2>&1
