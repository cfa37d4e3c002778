#!/bin/bash
# Mixtral decode with the fused QKV -> attention launch on its normed input: kernel test, Mixtral
# engine tests, then the bench alternating fused / two launches (POLYKEY_QKV_ATTN_FUSED=0)
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=gpurun_out
timeout -k 10 500 python -u -m pytest tests/kernels/test_attention.py tests/parallel/test_tp_gpu.py tests/parallel/test_ep_ipc_gpu.py -x -q --timeout 200 --timeout-method thread > $O/r6_mixf_test.log 2>&1
rc=$?; tail -3 $O/r6_mixf_test.log; [ $rc -eq 0 ] || exit $rc
rm -f $O/r6_mixf_ab.jsonl
for i in 1 2; do
  for f in 1 0; do
    POLYKEY_QKV_ATTN_FUSED=$f timeout -k 10 400 python bench.py --model mixtral-8x7b --steps 2 --warmup 1 > $O/r6_mixf_$f.json 2> $O/r6_mixf_$f.err || exit 1
    python3 -c "import json,sys; d=json.load(open('$O/r6_mixf_$f.json')); print(json.dumps({'qkv_attn_fused': $f, 'value': d['value'], 'ms_per_step': d['ms_per_step']}))" | tee -a $O/r6_mixf_ab.jsonl || exit 1
  done
done
