#!/bin/bash
# round 4, first box: smoke + GPU suite + headline bench, then per-rank decode-step times (tp_solo)
set -o pipefail
mkdir -p gpurun_out
bash tools/gpu/final_check.sh || exit 1
timeout -k 10 300 python -u tools/tp_solo.py --model llama3-8b --tp 1 > gpurun_out/solo_8b.json 2> gpurun_out/solo_8b.err || { tail -20 gpurun_out/solo_8b.err; exit 1; }
cat gpurun_out/solo_8b.json
timeout -k 10 400 python -u tools/tp_solo.py --model llama3-70b --tp 8 > gpurun_out/solo_70b_tp8.json 2> gpurun_out/solo_70b_tp8.err || { tail -20 gpurun_out/solo_70b_tp8.err; exit 1; }
cat gpurun_out/solo_70b_tp8.json
