#!/bin/bash
# round-end rehearsal: smoke(), the GPU suite, one headline bench run
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 1; }
echo smoke ok
timeout -k 10 700 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/gputest_final.log 2>&1 || { tail -30 gpurun_out/gputest_final.log; exit 1; }
tail -1 gpurun_out/gputest_final.log
timeout -k 10 400 python -u bench.py --steps 10 --warmup 2 > gpurun_out/bench_final.json 2> gpurun_out/bench_final.err || exit 1
cat gpurun_out/bench_final.json
