#!/bin/bash
# per-shape prefill GEMM selection (8-wave kernel for K >= 2N): tests, Mixtral and 70B-on-one-GPU benches
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=gpurun_out
timeout -k 10 300 python -u -m pytest tests/kernels/test_gemm_prefill.py tests/kernels/test_moe.py -x -q --timeout 120 --timeout-method thread > $O/r6_pe2_test.log 2>&1
rc=$?; tail -3 $O/r6_pe2_test.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py --model mixtral-8x7b --steps 3 --warmup 1 > $O/r6_bench_mixtral_b.json 2> $O/r6_bench_mixtral_b.err || exit 1
cat $O/r6_bench_mixtral_b.json
timeout -k 10 500 python bench.py --model llama3-70b --steps 1 --warmup 1 > $O/r6_bench_70b_tp1.json 2> $O/r6_bench_70b_tp1.err || { tail -30 $O/r6_bench_70b_tp1.err; exit 1; }
cat $O/r6_bench_70b_tp1.json
