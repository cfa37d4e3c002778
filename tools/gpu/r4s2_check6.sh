#!/bin/bash
# fused MLP (NT + LDS-prefetched down tiles) tests, e2e engine tests, headline bench, headline wave under a
# kernel trace (per-kernel step breakdown), PMC passes
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 500 python -u -m pytest -x -q --timeout 150 --timeout-method thread -m gpu tests/kernels/test_gemm_skinny.py \
  tests/e2e tests/parallel/test_tp_rank_death_gpu.py > gpurun_out/c6_tests.log 2>&1 || { tail -40 gpurun_out/c6_tests.log; exit 1; }
tail -1 gpurun_out/c6_tests.log
timeout -k 10 400 python bench.py --steps 10 --warmup 2 > gpurun_out/c6_bench.json 2> gpurun_out/c6_bench.err || { tail -30 gpurun_out/c6_bench.err; exit 1; }
cat gpurun_out/c6_bench.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_r4 -- \
  python3 $R/bench.py --steps 1 --warmup 1 > $R/gpurun_out/prof_r4.log 2>&1 || { tail -20 $R/gpurun_out/prof_r4.log; exit 1; }
cd $R
python3 tools/step_breakdown.py gpurun_out/prof_r4 gpurun_out/r4_8b_bench_step_breakdown.md || exit 1
find gpurun_out/prof_r4 -name '*kernel_stats.csv' -exec cp {} gpurun_out/r4_8b_bench_kernel_stats.csv \;
find gpurun_out/prof_r4 -name '*kernel_trace.csv' -delete
head -22 gpurun_out/r4_8b_bench_step_breakdown.md
bash $R/tools/gpu/fused_pmc.sh
