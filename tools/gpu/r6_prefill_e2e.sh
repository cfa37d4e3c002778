#!/bin/bash
# buffer-load prefill GEMM as the default: kernel tests + A/B vs hipBLASLt, then Mixtral and 70B-on-one-GPU benches
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=gpurun_out
timeout -k 10 300 python -u -m pytest tests/kernels/test_gemm_prefill.py tests/kernels/test_moe.py -x -q --timeout 120 --timeout-method thread > $O/r6_pe_test.log 2>&1
rc=$?; tail -3 $O/r6_pe_test.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 tools/prefill_gemm_ab.py 6 4 | tee $O/r6_pe_ab.txt || exit 1
timeout -k 10 400 python bench.py --model mixtral-8x7b --steps 3 --warmup 1 > $O/r6_bench_mixtral.json 2> $O/r6_bench_mixtral.err || exit 1
cat $O/r6_bench_mixtral.json
