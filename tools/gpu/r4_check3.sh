#!/bin/bash
# kernels + e2e + collective GPU tests, per-rank decode step (tp_solo) fused / unfused, headline bench
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/kernels tests/e2e \
  tests/parallel/test_tp_chain_gpu.py tests/parallel/test_custom_ar_gpu.py tests/parallel/test_tp8_shapes_gpu.py \
  > gpurun_out/r4c3_tests.log 2>&1 || { tail -40 gpurun_out/r4c3_tests.log; exit 1; }
tail -1 gpurun_out/r4c3_tests.log
rm -f gpurun_out/solo3.jsonl
for cfg in "llama3-8b 1" "llama3-70b 8"; do
  set -- $cfg
  timeout -k 10 300 python -u tools/tp_solo.py --model $1 --tp $2 >> gpurun_out/solo3.jsonl 2> gpurun_out/solo_$1.err || { tail -20 gpurun_out/solo_$1.err; exit 1; }
  POLYKEY_MLP_FUSED=0 POLYKEY_QKV_ATTN_FUSED=0 timeout -k 10 300 python -u tools/tp_solo.py --model $1 --tp $2 >> gpurun_out/solo3.jsonl 2>> gpurun_out/solo_$1.err || { tail -20 gpurun_out/solo_$1.err; exit 1; }
done
cat gpurun_out/solo3.jsonl
timeout -k 10 400 python -u bench.py --steps 10 --warmup 2 > gpurun_out/bench_r4c3.json 2> gpurun_out/bench_r4c3.err || exit 1
cat gpurun_out/bench_r4c3.json
