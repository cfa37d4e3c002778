#!/bin/bash
# 70B TP=8 per-rank decode chain options (in-launch attention merge, in-launch gate_up SiLU split,
# half-split QKV): correctness tests, then the per-rank step A/B and a per-(kernel, grid) profile
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 240 --timeout-method thread \
  "tests/kernels/test_phases.py::test_decode_inlaunch_partition_merge" \
  "tests/kernels/test_phases.py::test_gate_up_split_inlaunch_silu" tests/parallel/test_tp_chain_gpu.py \
  > $O/r5_tp_tests.log 2>&1; rc=$?; tail -3 $O/r5_tp_tests.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  for cfg in "0 0 0" "1 0 0" "0 1 0" "0 0 1" "1 1 1"; do
    set -- $cfg
    POLYKEY_DECODE_INLAUNCH_MERGE=$1 POLYKEY_GATE_UP_INLAUNCH=$2 POLYKEY_QKV_HALF=$3 timeout -k 10 200 \
      python3 tools/tp_solo.py --model llama3-70b --tp 8 --iters 30 | cut -c1-200 | tee -a $O/r5_tp_ab.jsonl || exit 1
  done
done
POLYKEY_DECODE_INLAUNCH_MERGE=1 timeout -k 10 200 python3 tools/tp_solo.py --model llama3-8b --tp 1 --iters 30 | cut -c1-200 | tee -a $O/r5_tp_ab.jsonl || exit 1
POLYKEY_DECODE_INLAUNCH_MERGE=0 timeout -k 10 200 python3 tools/tp_solo.py --model llama3-8b --tp 1 --iters 30 | cut -c1-200 | tee -a $O/r5_tp_ab.jsonl || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d /tmp/s70 -- python3 $R/tools/tp_solo.py --model llama3-70b \
  --tp 8 --iters 10 --eager > /tmp/s70.log 2>&1 || { tail -20 /tmp/s70.log; exit 1; }
python3 $R/tools/kgrid.py /tmp/s70 $R/$O/r5_70b_kgrid.md --per 13 > /dev/null
