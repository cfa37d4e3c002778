#!/bin/bash
# fused decode MLP launch: kernel tests, graph-captured decode step A/B, bench
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/kernels/test_gemm_skinny.py \
  -k "mlp_fused or rowscale or silu" > gpurun_out/mlp_tests.log 2>&1 || { tail -30 gpurun_out/mlp_tests.log; exit 1; }
tail -1 gpurun_out/mlp_tests.log
out=gpurun_out/mlp_ab.txt
: > $out
for cfg in f1 f0 f1b f0b; do
  v=0; [[ $cfg == f1* || $cfg == fi1* ]] && v=1; il=0; [[ $cfg == fi* ]] && il=1
  POLYKEY_MLP_FUSED=$v POLYKEY_MLP_INTERLEAVE=$il timeout -k 10 240 python tools/ab_decode.py --steps 128 --reps 3 --tag $cfg >> $out 2> gpurun_out/mlp_ab.err || { tail gpurun_out/mlp_ab.err; exit 1; }
done
cat $out
timeout -k 10 400 python -u bench.py --steps 10 --warmup 2 > gpurun_out/bench_mlp.json 2> gpurun_out/bench_mlp.err || exit 1
cat gpurun_out/bench_mlp.json
