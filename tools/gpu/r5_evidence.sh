#!/bin/bash
# round-5 evidence: per-kernel step breakdown of the headline bench wave, HBM fetch / MFMA counters
# of the 8B decode kernels (one counter group per pass)
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d /tmp/prof_r5 -- python3 $R/bench.py --steps 1 --warmup 1 \
  > /tmp/prof_r5.log 2>&1 || { tail -30 /tmp/prof_r5.log; exit 1; }
python3 $R/tools/step_breakdown.py /tmp/prof_r5 $R/gpurun_out/r5_8b_bench_step_breakdown.md > /dev/null || exit 1
head -16 $R/gpurun_out/r5_8b_bench_step_breakdown.md
run() {  # $1 tag, rest: counters
  local tag=$1; shift
  timeout -s KILL 240 rocprofv3 --pmc "$@" --output-format csv -d /tmp/pmc_$tag -- \
    python3 $R/tools/ab_decode.py --eager --steps 8 --reps 1 > /tmp/pmc_$tag.log 2>&1 \
    || { tail -60 /tmp/pmc_$tag.log > $R/gpurun_out/r5_pmc_$tag.err; tail -5 /tmp/pmc_$tag.log; return 1; }
  python3 $R/tools/pmc_summary.py /tmp/pmc_$tag $R/gpurun_out/r5_pmc_$tag.md > /dev/null || return 1
  head -14 $R/gpurun_out/r5_pmc_$tag.md
}
run fetch FETCH_SIZE GRBM_GUI_ACTIVE SQ_INSTS_MFMA && \
run mfma GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES
