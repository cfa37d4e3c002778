#!/bin/bash
# decode GEMM tests, then the graph-captured 8B decode step and the headline bench with the
# folded-norm QKV slabs from 64-row blocks at half the split (1) vs 128-row blocks (0)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/kernels/test_gemm_skinny.py tests/e2e/test_engine_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t_hq.log 2>&1 || exit 1
: > gpurun_out/ab_half_qkv.txt
for v in 0 1 0 1; do
  POLYKEY_HALF_QKV_SLABS=$v timeout -k 10 300 python tools/ab_decode.py --tag hq$v >> gpurun_out/ab_half_qkv.txt 2> gpurun_out/ab_hq.err || exit 1
done
for v in 0 1; do
  POLYKEY_HALF_QKV_SLABS=$v timeout -k 10 300 python bench.py > gpurun_out/bhq_$v.json 2> gpurun_out/bhq_$v.err || exit 1
  python -c "import json; d=json.load(open('gpurun_out/bhq_$v.json')); print('bench hq$v', d['value'], d['ms_per_step'])" >> gpurun_out/ab_half_qkv.txt
done
