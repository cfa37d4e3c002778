set -o pipefail
R=$GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/kernels/test_attention.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t_attn.log 2>&1 || exit 1
timeout -k 10 200 python tools/bench_prefill_attn.py > gpurun_out/prefill_attn.txt 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 -L > $R/gpurun_out/rocprof_counters.txt 2>&1 || true
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE --output-format csv -d $R/gpurun_out/pmc_attn -- python3 $R/tools/bench_prefill_attn.py > $R/gpurun_out/pmc_attn.log 2>&1
