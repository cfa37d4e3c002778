#!/bin/bash
# the production wide-decode rule (WIDE_MFMA_MIN_TILES row-weighted): GPU tests, 8B step at 384 / 448 / 512 rows
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
cd $R
rm -f $O/r6_wide_confirm.jsonl
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu \
  tests/e2e/test_engine_gpu.py -k "wide_decode or large_decode" > $O/r6_wide_confirm_tests.log 2>&1 || { tail -30 $O/r6_wide_confirm_tests.log; exit 1; }
tail -1 $O/r6_wide_confirm_tests.log
for b in 384 448 512; do
  timeout -k 10 200 python3 tools/tp_solo.py --model llama3-8b --tp 1 --batch $b --ctx 384 --iters 30 \
    | python3 -c 'import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(json.dumps({k: d[k] for k in ("batch","ms_per_step","wide_min_tiles")}))' \
    | tee -a $O/r6_wide_confirm.jsonl || exit 1
done
