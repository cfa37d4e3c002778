#!/bin/bash
# serving heap collector pauses: engine start with gc.freeze() + a larger gen-0 threshold
# (default) vs CPython's defaults (POLYKEY_GC_FREEZE=0), headline bench alternating, per-wave walls
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=gpurun_out
rm -f $O/r6_gc_ab.jsonl
for i in 1 2; do
  for g in 1 0; do
    POLYKEY_GC_FREEZE=$g POLYKEY_BENCH_TIMING=1 timeout -k 10 300 python3 bench.py --steps 20 --warmup 3 > $O/r6_gc_$g.log 2>&1 || { tail -20 $O/r6_gc_$g.log; exit 1; }
    python3 - "$O/r6_gc_$g.log" "$g" <<'PY' | tee -a $O/r6_gc_ab.jsonl
import json, re, sys
txt = open(sys.argv[1]).read()
walls = [float(x) for x in re.findall(r"\[wave\] wall ([0-9.]+) ms", txt)]
line = json.loads([l for l in txt.splitlines() if l.startswith('{"metric"')][-1])
timed = walls[-20:]
print(json.dumps({"gc_freeze": int(sys.argv[2]), "value": line["value"], "ms_per_step": line["ms_per_step"],
                  "wave_ms_min": min(timed), "wave_ms_max": max(timed), "waves_over_min_plus_20ms": sum(w > min(timed) + 20 for w in timed)}))
PY
  done
done
