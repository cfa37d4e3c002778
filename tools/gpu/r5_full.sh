#!/bin/bash
# round-5 check: the whole GPU suite, smoke, the driver's bench (+ a prefill-budget A/B), and the
# 70B per-rank attention partition A/B
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/r5_gpu_suite.log 2>&1
rc=$?; tail -4 $O/r5_gpu_suite.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" 2>&1 | tail -2 || exit 1
for f in 256 0; do
  POLYKEY_DECODE_FILL=$f timeout -k 10 200 python3 tools/tp_solo.py --model llama3-70b --tp 8 --iters 30 | cut -c1-160 | sed "s/^{/{\"fill\": $f, /" | tee -a $O/r5_fill.jsonl || exit 1
done
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/r5_bench.log 2>&1 || { tail -20 $O/r5_bench.log; exit 1; }
tail -1 $O/r5_bench.log | tee $O/r5_bench.json
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 --max-batched-tokens 16384 > $O/r5_bench_16k.log 2>&1 || { tail -20 $O/r5_bench_16k.log; exit 1; }
tail -1 $O/r5_bench_16k.log | tee $O/r5_bench_16k.json
