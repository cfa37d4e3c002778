#!/bin/bash
# headline bench twice (plain, then with the per-wave host timing breakdown on stderr)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --steps 5 > gpurun_out/bench.json 2> gpurun_out/bench.err && \
POLYKEY_BENCH_TIMING=1 timeout -k 10 300 python bench.py --steps 5 > gpurun_out/bench_t.json 2> gpurun_out/bench_t.err
