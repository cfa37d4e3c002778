#!/bin/bash
# decode attention at 3 waves / SIMD (__launch_bounds__(256, 3)): tests, per-rank step at 64-512 rows
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 240 --timeout-method thread \
  tests/kernels/test_phases.py tests/kernels/test_attention.py \
  > $O/r5_occ_tests.log 2>&1; rc=$?; tail -2 $O/r5_occ_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 tools/attn70_probe.py --heads 32,8 | cut -c1-100 | head -6 | tee $O/r5_occ_probe.jsonl || exit 1
for b in 64 256 512; do
  timeout -k 10 200 python3 tools/tp_solo.py --model llama3-8b --tp 1 --batch $b --iters 20 | cut -c1-130 | tee -a $O/r5_occ.jsonl || exit 1
done
timeout -k 10 200 python3 tools/tp_solo.py --model llama3-70b --tp 8 --iters 30 | cut -c1-130 | tee -a $O/r5_occ.jsonl || exit 1
