#!/bin/bash
# PMC passes at gate_up: the current 4-wave kernel (6) vs hipBLASLt -- L1 / address-unit stalls, waits, MFMA busy
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
pass() {  # $1 tag, rest: counters
  local tag=$1; shift
  timeout -s KILL 90 rocprofv3 --pmc "$@" --output-format csv -d /tmp/pmc_$tag -- python3 $R/tools/pg_pmc_driver.py 6 \
    > /tmp/pmc_$tag.log 2>&1 || { tail -30 /tmp/pmc_$tag.log > $R/gpurun_out/r6_pg_pmc_$tag.err; tail -5 /tmp/pmc_$tag.log; return 1; }
  python3 $R/tools/pmc_summary.py /tmp/pmc_$tag $R/gpurun_out/r6_pg_pmc_$tag.md > /dev/null || return 1
  cat $R/gpurun_out/r6_pg_pmc_$tag.md
}
pass b TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VMEM_RD && \
pass c TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES && \
pass d SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_VMEM
