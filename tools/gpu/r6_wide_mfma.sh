#!/bin/bash
# wide decode on the prefill MFMA GEMM (models/llama.py WIDE_MFMA_MIN_TILES): GPU tests, the 8B
# decode step at 256 / 384 / 512 rows with and without it (graph replay), then the 256 / 512-client
# bench of the headline config
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
cd $R
rm -f $O/r6_wide_mfma.jsonl
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu \
  tests/e2e/test_engine_gpu.py -k "wide_decode or large_decode or packed_only" > $O/r6_wide_mfma_tests.log 2>&1 || { tail -30 $O/r6_wide_mfma_tests.log; exit 1; }
tail -2 $O/r6_wide_mfma_tests.log
for b in 256 384 512; do
  for t in 224 1000000000 224; do
    timeout -k 10 200 python3 tools/tp_solo.py --model llama3-8b --tp 1 --batch $b --ctx 384 --iters 20 --wide-min-tiles $t \
      | python3 -c 'import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(json.dumps({k: d[k] for k in ("batch","ms_per_step","wide_min_tiles")}))' \
      | tee -a $O/r6_wide_mfma.jsonl || exit 1
  done
done
for c in 256 512; do
  timeout -k 10 400 python3 -u bench.py --steps 1 --warmup 1 --concurrency $c > $O/r6_wide_conc_$c.log 2>&1 || { tail -30 $O/r6_wide_conc_$c.log; exit 1; }
  grep '^{"metric"' $O/r6_wide_conc_$c.log | cut -c1-400 | tee -a $O/r6_wide_mfma.jsonl
done
