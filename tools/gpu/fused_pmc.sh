#!/bin/bash
# PMC counters of the 8B decode step kernels (eager engine, 64 sequences): the fused launches'
# HBM bytes and MFMA activity next to the plain decode GEMMs.  One counter group per pass.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE GRBM_GUI_ACTIVE SQ_INSTS_MFMA SQ_BUSY_CYCLES --output-format csv \
  -d $R/gpurun_out/pmc_fused1 -- python3 $R/tools/ab_decode.py --eager --steps 8 --reps 1 > $R/gpurun_out/pmc_fused1.log 2>&1 && \
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES --output-format csv \
  -d $R/gpurun_out/pmc_fused2 -- python3 $R/tools/ab_decode.py --eager --steps 8 --reps 1 > $R/gpurun_out/pmc_fused2.log 2>&1 && \
cd $R && python3 tools/pmc_summary.py gpurun_out/pmc_fused1 gpurun_out/r3_fused_pmc1.md > /dev/null && \
python3 tools/pmc_summary.py gpurun_out/pmc_fused2 gpurun_out/r3_fused_pmc2.md > /dev/null && \
find gpurun_out/pmc_fused1 gpurun_out/pmc_fused2 -name '*counter_collection.csv' -delete; \
head -20 gpurun_out/r3_fused_pmc1.md; head -20 gpurun_out/r3_fused_pmc2.md
