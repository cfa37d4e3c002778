#!/bin/bash
# EP IPC tests (decode + prefill-sized regions), EP=2 vs EP=1 bench, one gateway run with timing
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 500 --timeout-method thread tests/parallel/test_ep_ipc_gpu.py \
  tests/kernels/test_moe.py > gpurun_out/ep_tests.log 2>&1 || { tail -40 gpurun_out/ep_tests.log; exit 1; }
tail -2 gpurun_out/ep_tests.log
rm -f gpurun_out/ep_bench.jsonl
bash tools/gpu/ep_bench.sh || exit 1
POLYKEY_BENCH_TIMING=1 GPU_MAX_HW_QUEUES=1 timeout -k 10 420 python -u bench.py --gpus 4 --steps 2 --warmup 1 \
  --num-kv-blocks 1300 --frontend gateway > gpurun_out/gw_timing.log 2>&1
grep "\[gateway\]\|^{" gpurun_out/gw_timing.log | cut -c1-300
grep "\[wave\]" gpurun_out/gw_timing.log | head -8
