#!/bin/bash
# PMC counters of the 8B decode step kernels (eager engine, 64 sequences): the fused launches'
# HBM bytes and MFMA activity next to the plain decode GEMMs.  One counter group per pass; raw
# rocprofv3 output stays in /tmp on the box, the summaries (and a failed pass's log) come back.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
run() {  # $1 tag, rest: counters
  local tag=$1; shift
  timeout -s KILL 240 rocprofv3 --pmc "$@" --output-format csv -d /tmp/pmc_$tag -- \
    python3 $R/tools/ab_decode.py --eager --steps 8 --reps 1 > /tmp/pmc_$tag.log 2>&1 \
    || { tail -60 /tmp/pmc_$tag.log > $R/gpurun_out/r4_fused_pmc_$tag.err; tail -5 /tmp/pmc_$tag.log; return 1; }
  python3 $R/tools/pmc_summary.py /tmp/pmc_$tag $R/gpurun_out/r4_fused_pmc_$tag.md > /dev/null || return 1
  head -16 $R/gpurun_out/r4_fused_pmc_$tag.md
}
# (FETCH_SIZE with SQ_VALU_MFMA_BUSY_CYCLES in one pass segfaulted the profiled process once: separate
# passes, and the first failed pass ends the script)
run a FETCH_SIZE GRBM_GUI_ACTIVE SQ_INSTS_MFMA && \
run b GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_WAVES SQ_LDS_BANK_CONFLICT && \
run c GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES
