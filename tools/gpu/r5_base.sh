#!/bin/bash
# round-5 baseline: per-rank decode step (tools/tp_solo.py) kernel stats, 70B TP=8 serving chain + 8B TP=1
set -o pipefail
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
prof() {  # tag, env..., -- args
  local tag=$1; shift
  env "$@" timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/solo_$tag -- \
    python3 $R/tools/tp_solo.py $SOLO_ARGS > /tmp/solo_$tag.log 2>&1 || { tail -20 /tmp/solo_$tag.log; return 1; }
  python3 $R/tools/kstats.py /tmp/solo_$tag $R/gpurun_out/r5_solo_${tag}_kstats.md 24 > /dev/null
  tail -1 /tmp/solo_$tag.log | tee -a $R/gpurun_out/r5_base.jsonl
}
cd $R && timeout -k 10 200 python3 tools/tp_solo.py --model llama3-70b --tp 8 | tee -a gpurun_out/r5_base.jsonl && \
timeout -k 10 200 python3 tools/tp_solo.py --model llama3-8b --tp 1 | tee -a gpurun_out/r5_base.jsonl && cd /tmp && \
SOLO_ARGS="--model llama3-70b --tp 8 --iters 10 --eager" prof 70b_tp8_eager && \
SOLO_ARGS="--model llama3-8b --tp 1 --iters 10 --eager" prof 8b_eager
