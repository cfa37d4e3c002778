#!/bin/bash
# round 6 check after the variant prune: the whole GPU suite, smoke, the 70B TP=8 rank (local-half
# and loopback collectives) and the driver's 1-GPU bench
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=gpurun_out
TAG=${1:-a}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/r6_gpu_suite_$TAG.log 2>&1
rc=$?; tail -4 $O/r6_gpu_suite_$TAG.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 150 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/r6_smoke_$TAG.log 2>&1 || { tail -20 $O/r6_smoke_$TAG.log; exit 1; }
tail -2 $O/r6_smoke_$TAG.log
for c in solo loopback; do
  timeout -k 10 200 python3 tools/tp_solo.py --model llama3-70b --tp 8 --iters 30 --car $c | cut -c1-200 | tee -a $O/r6_tp8_$TAG.jsonl || exit 1
done
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/r6_bench_$TAG.log 2>&1 || { tail -20 $O/r6_bench_$TAG.log; exit 1; }
tail -1 $O/r6_bench_$TAG.log | tee $O/r6_bench_$TAG.json
