#!/bin/bash
# prefill-GEMM / MoE tests, then the Mixtral bench with prefill GEMM variant 2 vs 4 (alternating)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/kernels/test_gemm_prefill.py tests/kernels/test_moe.py tests/e2e/test_engine_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t_mix.log 2>&1 || exit 1
: > gpurun_out/mix_ab.txt
for v in 2 4 2 4; do
  POLYKEY_PREFILL_GEMM_VARIANT=$v timeout -k 10 300 python bench.py --model mixtral-8x7b --steps 2 --warmup 1 > gpurun_out/bm_$v.json 2> gpurun_out/bm_$v.err || exit 1
  python -c "import json; d=json.load(open('gpurun_out/bm_$v.json')); print('variant $v', d['value'], d['ms_per_step'], d['p50_e2e_latency_ms'])" >> gpurun_out/mix_ab.txt
done
