#!/bin/bash
# gate_up at 384-512 decode rows on the MFMA GEMM (224+ tiles, production) vs hipBLASLt with the LM head
# on the MFMA GEMM in both (--wide-min-tiles 500), 8B decode step, graph replay, alternating
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
cd $R
rm -f $O/r6_wide384.jsonl
for b in 384 448 512; do
  for t in 224 500 224 500; do
    timeout -k 10 200 python3 tools/tp_solo.py --model llama3-8b --tp 1 --batch $b --ctx 384 --iters 30 --wide-min-tiles $t \
      | python3 -c 'import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(json.dumps({k: d[k] for k in ("batch","ms_per_step","wide_min_tiles")}))' \
      | tee -a $O/r6_wide384.jsonl || exit 1
  done
done
