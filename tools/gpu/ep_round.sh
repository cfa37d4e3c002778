#!/bin/bash
# grouped row-tile kernels + EP tests, the EP=2 kernel-trace profile, EP bench A/B, gateway A/B
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 500 --timeout-method thread tests/kernels/test_moe.py \
  tests/kernels/test_gemm_skinny.py -k "row_tiles or grouped" tests/parallel/test_ep_ipc_gpu.py > gpurun_out/ep_tests.log 2>&1 \
  || { tail -40 gpurun_out/ep_tests.log; exit 1; }
tail -2 gpurun_out/ep_tests.log
bash tools/gpu/ep_prof.sh && rm -f gpurun_out/ep_bench.jsonl gpurun_out/gateway_ab.jsonl && bash tools/gpu/ep_bench.sh \
  && bash tools/gpu/gateway_ab.sh
