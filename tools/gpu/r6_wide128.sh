#!/bin/bash
# 8B per-rank decode step at 128 rows: graph-replay time, then a per-(kernel, grid) profile (eager)
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
cd $R
timeout -k 10 200 python3 tools/tp_solo.py --model llama3-8b --tp 1 --batch 128 --ctx 384 --iters 20 | cut -c1-200 | tee $O/r6_wide128.jsonl || exit 1
cd /tmp && export TMPDIR=/tmp
rm -rf /tmp/w128
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d /tmp/w128 -- python3 $R/tools/tp_solo.py --model llama3-8b --tp 1 --batch 128 --ctx 384 --iters 10 --eager > $O/r6_wide128_prof.log 2>&1 || exit 1
python3 $R/tools/kgrid.py /tmp/w128 $O/r6_wide128_kgrid.md --per 13 > /dev/null || exit 1
head -24 $O/r6_wide128_kgrid.md | cut -c1-220
