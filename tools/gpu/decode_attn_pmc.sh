#!/bin/bash
# PMC counters of the decode attention kernels at the bench shape (tools/attn_lab.py, ctx 384)
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INST_LEVEL_VMEM SQ_INSTS_VMEM_RD SQ_LEVEL_WAVES GRBM_GUI_ACTIVE --output-format csv -d $R/gpurun_out/pmc_dattn1 -- python3 $R/tools/attn_lab.py --ctx 384 --iters 20 > $R/gpurun_out/pmc_dattn1.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE GRBM_GUI_ACTIVE SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU --output-format csv -d $R/gpurun_out/pmc_dattn2 -- python3 $R/tools/attn_lab.py --ctx 384 --iters 20 > $R/gpurun_out/pmc_dattn2.log 2>&1
