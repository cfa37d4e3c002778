#!/bin/bash
# per-kernel stats of the per-rank decode step (tools/tp_solo.py) under rocprofv3:
# 70B TP=8 shard with / without the fused launches, 8B TP=1 for reference
set -o pipefail
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
prof() {  # tag, env..., -- args
  local tag=$1; shift
  env "$@" timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/solo_$tag -- \
    python3 $R/tools/tp_solo.py $SOLO_ARGS > /tmp/solo_$tag.log 2>&1 || { tail -20 /tmp/solo_$tag.log; return 1; }
  python3 $R/tools/kstats.py /tmp/solo_$tag $R/gpurun_out/solo_${tag}_kstats.md 24 | head -30
  tail -1 /tmp/solo_$tag.log
}
SOLO_ARGS="--model llama3-70b --tp 8 --iters 10" prof 70b_tp8_fused POLYKEY_MLP_FUSED=1 && \
SOLO_ARGS="--model llama3-70b --tp 8 --iters 10" prof 70b_tp8_unfused POLYKEY_MLP_FUSED=0 POLYKEY_QKV_ATTN_FUSED=0 && \
SOLO_ARGS="--model llama3-8b --tp 1 --iters 10" prof 8b_fused POLYKEY_MLP_FUSED=1
