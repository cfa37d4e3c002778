#!/bin/bash
# round 4: re-check the TP=8 noise-band tests (numbers printed), the headline bench, and the
# per-rank decode step (tp_solo) of 8B TP=1 and 70B TP=8 with / without the fused launches
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread tests/parallel/test_tp8_shapes_gpu.py \
  tests/kernels/test_gemm_skinny.py::test_fused_err_word_plumbing tests/parallel/test_tp_chain_gpu.py \
  "tests/e2e/test_engine_gpu.py::test_fused_handoff_timeout_falls_back_to_two_launches" > gpurun_out/r4c2_tests.log 2>&1 \
  || { tail -40 gpurun_out/r4c2_tests.log; exit 1; }
grep -o '"ref_logits_row_mean_abs_diff[^}]*' gpurun_out/r4c2_tests.log | cut -c1-400
tail -2 gpurun_out/r4c2_tests.log
timeout -k 10 400 python -u bench.py --steps 10 --warmup 2 > gpurun_out/bench_r4c2.json 2> gpurun_out/bench_r4c2.err || exit 1
cat gpurun_out/bench_r4c2.json
for cfg in "llama3-8b 1" "llama3-70b 8"; do
  set -- $cfg
  timeout -k 10 300 python -u tools/tp_solo.py --model $1 --tp $2 >> gpurun_out/solo.jsonl 2> gpurun_out/solo_$1.err || { tail -20 gpurun_out/solo_$1.err; exit 1; }
  POLYKEY_MLP_FUSED=0 POLYKEY_QKV_ATTN_FUSED=0 timeout -k 10 300 python -u tools/tp_solo.py --model $1 --tp $2 >> gpurun_out/solo.jsonl 2>> gpurun_out/solo_$1.err || { tail -20 gpurun_out/solo_$1.err; exit 1; }
done
cat gpurun_out/solo.jsonl
