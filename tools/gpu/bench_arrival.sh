# arrival-window variants of the headline bench (same box)
set -o pipefail
: > gpurun_out/arrival_ab.txt
for v in "step:8:2" "burst:8:2" "burst:30:3" "step:0:2" "step:8:2"; do
  IFS=: read fill win gap <<< "$v"
  POLYKEY_ARRIVAL_FILL=$fill POLYKEY_ARRIVAL_WINDOW_MS=$win POLYKEY_ARRIVAL_GAP_MS=$gap timeout -k 10 300 python bench.py > gpurun_out/b_arr.json 2>/dev/null || exit 1
  echo "$v $(cat gpurun_out/b_arr.json)" >> gpurun_out/arrival_ab.txt
done
