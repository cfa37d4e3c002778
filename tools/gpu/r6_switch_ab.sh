#!/bin/bash
# GIL switch interval of the serving process (engine thread vs event loop): 2 ms (default) vs 0.5 ms,
# headline bench alternating, per-wave RPC legs
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=gpurun_out
rm -f $O/r6_switch_ab.jsonl
for i in 1 2; do
  for g in 2 0.5; do
    POLYKEY_SWITCH_INTERVAL_MS=$g POLYKEY_BENCH_TIMING=1 timeout -k 10 300 python3 bench.py --steps 15 --warmup 3 > $O/r6_switch_$g.log 2>&1 || { tail -20 $O/r6_switch_$g.log; exit 1; }
    python3 - "$O/r6_switch_$g.log" "$g" <<'PY' | tee -a $O/r6_switch_ab.jsonl
import json, re, sys, statistics
txt = open(sys.argv[1]).read()
walls = [float(x) for x in re.findall(r"\[wave\] wall ([0-9.]+) ms", txt)][-15:]
legs = [float(x) for x in re.findall(r"request leg ([0-9.]+)/", txt)][-15:]
outs = [float(x) for x in re.findall(r"response leg ([0-9.]+)/", txt)][-15:]
line = json.loads([l for l in txt.splitlines() if l.startswith('{"metric"')][-1])
print(json.dumps({"switch_ms": float(sys.argv[2]), "value": line["value"], "wave_ms_median": statistics.median(walls),
                  "request_leg_p50_median": statistics.median(legs), "response_leg_p50_median": statistics.median(outs)}))
PY
  done
done
