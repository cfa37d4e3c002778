#!/bin/bash
# Kernel traces of the Mixtral DP-attention + EP=2 bench, both ranks on ONE MI355X, each rank
# launched directly (no torchrun) under rocprofv3 --kernel-trace; merged report via tp_gaps.py.
cd /tmp && export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/ep_prof
rm -rf $OUT && mkdir -p $OUT
PORT=$((29500 + RANDOM % 1000))
EP=${EP:-2}
pids=()
for r in $(seq 0 $((EP - 1))); do
  RANK=$r LOCAL_RANK=$r WORLD_SIZE=$EP LOCAL_WORLD_SIZE=$EP MASTER_ADDR=127.0.0.1 MASTER_PORT=$PORT GPU_MAX_HW_QUEUES=1 \
    timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $OUT/trace_r$r -- \
    python -u bench.py --gpus $EP --tp 1 --ep $EP --model mixtral-8x7b --steps 1 --warmup 1 --num-kv-blocks 2048 \
    > $OUT/rank$r.log 2>&1 &
  pids+=($!)
done
rc=0
for p in "${pids[@]}"; do wait $p || rc=$?; done
echo "ranks rc=$rc"
grep -h '^{"metric"' $OUT/rank0.log || tail -20 $OUT/rank0.log
python tools/tp_gaps.py $(for r in $(seq 0 $((EP - 1))); do echo -n "$OUT/trace_r$r "; done) --out $OUT/gaps.md > /dev/null \
  && head -40 $OUT/gaps.md
find $OUT -name '*.csv' -size +20M -delete
exit $rc
