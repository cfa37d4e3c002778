# PMC counters of the prefill-attention kernels on the 2 x 4096 causal case (one pass per kernel)
set -o pipefail
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
for impl in 1 2; do
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_ANY GRBM_GUI_ACTIVE --output-format csv -d $R/gpurun_out/pmc_attn_i$impl -- python3 $R/tools/attn_case.py $impl > $R/gpurun_out/pmc_attn_i$impl.log 2>&1 || exit 1
done
