#!/bin/bash
# fused QKV -> decode attention launch: kernel tests, graph-captured decode step A/B, bench
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/kernels/test_attention.py \
  tests/kernels/test_gemm_skinny.py -k "qkv_attn_fused or decode_from_qkv or mlp_fused or rowscale" > gpurun_out/qa_tests.log 2>&1 || { tail -30 gpurun_out/qa_tests.log; exit 1; }
tail -1 gpurun_out/qa_tests.log
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/e2e > gpurun_out/qa_e2e.log 2>&1 || { tail -30 gpurun_out/qa_e2e.log; exit 1; }
tail -1 gpurun_out/qa_e2e.log
out=gpurun_out/qa_ab.txt
: > $out
for cfg in f1 f0 f1b f0b; do
  v=0; [[ $cfg == f1* ]] && v=1
  POLYKEY_QKV_ATTN_FUSED=$v timeout -k 10 240 python tools/ab_decode.py --steps 128 --reps 3 --tag $cfg >> $out 2> gpurun_out/qa_ab.err || { tail gpurun_out/qa_ab.err; exit 1; }
done
cat $out
timeout -k 10 400 python -u bench.py --steps 10 --warmup 2 > gpurun_out/bench_qa.json 2> gpurun_out/bench_qa.err || exit 1
cat gpurun_out/bench_qa.json
