#!/bin/bash
# RoPE through one non-contracting helper in every kernel + the early cos / sin request
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=gpurun_out
timeout -k 10 500 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/kernels/test_attention.py tests/kernels/test_phases.py \
  tests/kernels/test_gemm_skinny.py tests/parallel/test_tp_chain_gpu.py tests/e2e/test_engine_gpu.py > $O/r5_cos_tests.log 2>&1; rc=$?; tail -2 $O/r5_cos_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 tools/attn70_probe.py | cut -c1-100 | head -6 | tee $O/r5_attn70_probe4.jsonl || exit 1
for i in 1 2; do
  timeout -k 10 200 python3 tools/tp_solo.py --model llama3-70b --tp 8 --iters 30 | cut -c1-110 | tee -a $O/r5_cos.jsonl || exit 1
  timeout -k 10 200 python3 tools/tp_solo.py --model llama3-8b --tp 1 --iters 30 | cut -c1-110 | tee -a $O/r5_cos.jsonl || exit 1
done
