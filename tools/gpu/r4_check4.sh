#!/bin/bash
# attention / fused kernels + collectives tests, per-rank 70B TP=8 decode step fused / unfused + kernel stats
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/kernels/test_attention.py \
  tests/parallel/test_tp_chain_gpu.py tests/parallel/test_custom_ar_gpu.py tests/parallel/test_tp8_shapes_gpu.py \
  > gpurun_out/r4c4_tests.log 2>&1 || { tail -40 gpurun_out/r4c4_tests.log; exit 1; }
tail -1 gpurun_out/r4c4_tests.log
rm -f gpurun_out/solo4.jsonl
timeout -k 10 300 python -u tools/tp_solo.py --model llama3-70b --tp 8 >> gpurun_out/solo4.jsonl 2> gpurun_out/solo4.err || { tail -20 gpurun_out/solo4.err; exit 1; }
POLYKEY_MLP_FUSED=0 POLYKEY_QKV_ATTN_FUSED=0 timeout -k 10 300 python -u tools/tp_solo.py --model llama3-70b --tp 8 >> gpurun_out/solo4.jsonl 2>> gpurun_out/solo4.err || { tail -20 gpurun_out/solo4.err; exit 1; }
POLYKEY_MLP_FUSED=1 POLYKEY_QKV_ATTN_FUSED=0 timeout -k 10 300 python -u tools/tp_solo.py --model llama3-70b --tp 8 >> gpurun_out/solo4.jsonl 2>> gpurun_out/solo4.err || { tail -20 gpurun_out/solo4.err; exit 1; }
cat gpurun_out/solo4.jsonl
SOLO_ARGS="--model llama3-70b --tp 8 --iters 10" bash -c 'cd /tmp && export TMPDIR=/tmp && R=$GRAFT_REPO_ROOT && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/solo_f -- python3 $R/tools/tp_solo.py $SOLO_ARGS > /tmp/solo_f.log 2>&1 && python3 $R/tools/kstats.py /tmp/solo_f $R/gpurun_out/solo_70b_tp8_fused2_kstats.md 14 | grep -v "distribution\|elementwise\|CatArray"'
