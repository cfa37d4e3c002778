#!/bin/bash
# in-launch phases (phase.h residual phase, decode_fused.hip o-projection phase) and the
# overlapped TP collective: kernel + e2e bit-identity tests, then the per-rank decode step A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/kernels/test_phases.py \
  "tests/kernels/test_gemm_skinny.py::test_mlp_fused_matches_two_launches" \
  "tests/kernels/test_attention.py::test_qkv_attn_fused_matches_two_launches" \
  "tests/e2e/test_engine_gpu.py::test_residual_phase_decode_is_bit_identical" \
  "tests/e2e/test_engine_gpu.py::test_fused_handoff_timeout_falls_back_to_two_launches" \
  tests/parallel/test_custom_ar_gpu.py tests/parallel/test_tp_chain_gpu.py > $O/r5_phase_tests.log 2>&1
rc=$?; tail -5 $O/r5_phase_tests.log; [ $rc -eq 0 ] || exit $rc
for cfg in "0 0" "1 0" "1 1" "0 0" "1 0" "1 1"; do
  set -- $cfg
  POLYKEY_RES_PHASE=$1 POLYKEY_O_PHASE=$2 timeout -k 10 200 python3 tools/tp_solo.py --model llama3-8b --tp 1 | sed "s/^{/{\"res_phase\": $1, \"o_phase\": $2, /" | tee -a $O/r5_phase_ab.jsonl || exit 1
done
for q in 4 1; do
  POLYKEY_QKV_MIN_KV=$q timeout -k 10 200 python3 tools/tp_solo.py --model llama3-70b --tp 8 | sed "s/^{/{\"qkv_min_kv\": $q, /" | tee -a $O/r5_phase_ab.jsonl || exit 1
done
