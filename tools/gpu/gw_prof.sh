#!/bin/bash
# SO_REUSEPORT gateway, 4 ranks on ONE MI355X, each rank launched directly under rocprofv3
# --kernel-trace: per-rank GPU busy over time (tools/busy_timeline.py) to tell a GPU-bound slow
# wave from a host-starved one.
cd /tmp && export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/gw_prof
rm -rf $OUT && mkdir -p $OUT
PORT=$((29500 + RANDOM % 1000))
N=4
pids=()
for r in $(seq 0 $((N - 1))); do
  RANK=$r LOCAL_RANK=$r WORLD_SIZE=$N LOCAL_WORLD_SIZE=$N MASTER_ADDR=127.0.0.1 MASTER_PORT=$PORT GPU_MAX_HW_QUEUES=1 \
    POLYKEY_BENCH_TIMING=1 timeout -k 10 500 rocprofv3 --kernel-trace --output-format csv -d $OUT/trace_r$r -- \
    python -u bench.py --gpus $N --steps 2 --warmup 1 --num-kv-blocks 1300 --frontend ${FE:-gateway} \
    > $OUT/rank$r.log 2>&1 &
  pids+=($!)
done
rc=0
for p in "${pids[@]}"; do wait $p || rc=$?; done
echo "ranks rc=$rc"
grep -h '^{"metric"' $OUT/rank0.log | cut -c1-200
grep -h "\[wave\]\|\[gateway\]" $OUT/rank*.log | cut -c1-200
python tools/busy_timeline.py $OUT/trace_r0 $OUT/trace_r1 $OUT/trace_r2 $OUT/trace_r3 --bin-ms 1000 --out $OUT/busy.md > /dev/null
cat $OUT/busy.md
python - <<'PY'
import csv, glob
for r in range(4):
    f = glob.glob(f"gpurun_out/gw_prof/trace_r{r}/**/*kernel_trace.csv", recursive=True)[0]
    rows = list(csv.DictReader(open(f)))
    t0 = min(int(x["Start_Timestamp"]) for x in rows)
    long = [x for x in rows if int(x["End_Timestamp"]) - int(x["Start_Timestamp"]) > 20_000_000]
    print(f"rank {r}: {len(rows)} kernels, {len(long)} longer than 20 ms")
    for x in long[:12]:
        s, e = int(x["Start_Timestamp"]), int(x["End_Timestamp"])
        print(f"  t={(s - t0) / 1e9:8.3f}s dur={(e - s) / 1e6:9.1f}ms queue={x.get('Queue_Id', '?')} "
              f"stream={x.get('Stream_Id', '?')} grid={x.get('Grid_Size', '?')} {x['Kernel_Name'][:110]}")
PY
find $OUT -name '*.csv' -delete
exit $rc
