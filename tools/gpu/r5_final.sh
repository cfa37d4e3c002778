#!/bin/bash
# end-of-round check: the whole GPU suite, smoke, the driver's bench, and the 70B TP=8 rank with
# its collectives as the local half and as the real kernels on a loopback group
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=gpurun_out
timeout -k 10 800 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/r5_gpu_suite_e.log 2>&1
rc=$?; tail -4 $O/r5_gpu_suite_e.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" 2>&1 | tail -2 || exit 1
for c in solo loopback; do
  timeout -k 10 200 python3 tools/tp_solo.py --model llama3-70b --tp 8 --iters 30 --car $c | cut -c1-160 | tee -a $O/r5_final_tp8_e.jsonl || exit 1
done
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/r5_bench_e.log 2>&1 || { tail -20 $O/r5_bench_e.log; exit 1; }
tail -1 $O/r5_bench_e.log | tee $O/r5_bench_e.json
