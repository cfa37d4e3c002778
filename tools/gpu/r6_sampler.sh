#!/bin/bash
# sampler first pass split over 8 workgroups per row: tests, smoke, then the headline wave per kernel
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=$R/gpurun_out
timeout -k 10 300 python -u -m pytest tests/kernels/test_sampler.py tests/e2e/test_engine_gpu.py -x -q --timeout 200 --timeout-method thread > $O/r6_sampler_test.log 2>&1
rc=$?; tail -3 $O/r6_sampler_test.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 150 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/r6_sampler_smoke.log 2>&1 || { tail -20 $O/r6_sampler_smoke.log; exit 1; }
tail -1 $O/r6_sampler_smoke.log
cd /tmp && export TMPDIR=/tmp
rm -rf /tmp/ws
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d /tmp/ws -- python3 $R/bench.py --steps 1 --warmup 1 > $O/r6_sampler_bench.log 2>&1 || { tail -20 $O/r6_sampler_bench.log; exit 1; }
python3 $R/tools/step_breakdown.py /tmp/ws $O/r6_sampler_breakdown.md > /dev/null || exit 1
head -20 $O/r6_sampler_breakdown.md
