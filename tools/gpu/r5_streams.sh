#!/bin/bash
# two-stream concurrency in one process: without and with the kernel tracer
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=gpurun_out
timeout -k 10 120 python3 tools/stream_concurrency_probe.py | tee $O/r5_streams.jsonl || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d /tmp/sc -- python3 $R/tools/stream_concurrency_probe.py \
  | tee -a $R/$O/r5_streams.jsonl || exit 1
python3 $R/tools/overlap_report.py /tmp/sc $R/$O/r5_streams_overlap.md | head -12
