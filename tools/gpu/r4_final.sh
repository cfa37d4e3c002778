#!/bin/bash
# round-4 end-of-session check on one MI355X: GPU suite, smoke(), headline bench (10 waves), the
# concurrency sweep 128 / 256 / 512, the 70B TP=8 per-rank step, PMC MFMA pass
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 700 python -u -m pytest -q --timeout 150 --timeout-method thread -m gpu tests \
  > gpurun_out/final_gpu_suite.log 2>&1; rc=$?
tail -8 gpurun_out/final_gpu_suite.log
[ $rc -eq 124 ] || [ $rc -eq 137 ] && exit 1
grep -q "Fatal Python error\|Segmentation fault\|core dumped" gpurun_out/final_gpu_suite.log && exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/final_smoke.log 2>&1 || { tail -20 gpurun_out/final_smoke.log; exit 1; }
tail -2 gpurun_out/final_smoke.log
timeout -k 10 400 python bench.py --steps 10 --warmup 2 > gpurun_out/final_bench.json 2> gpurun_out/final_bench.err || { tail -30 gpurun_out/final_bench.err; exit 1; }
cat gpurun_out/final_bench.json
timeout -k 10 400 python -u tools/tp_solo.py --model llama3-70b --tp 8 --iters 20 > gpurun_out/final_tp8_solo.log 2>&1 || { tail -20 gpurun_out/final_tp8_solo.log; exit 1; }
tail -1 gpurun_out/final_tp8_solo.log
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 240 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES --output-format csv -d /tmp/pmc_c -- \
  python3 $R/tools/ab_decode.py --eager --steps 8 --reps 1 > /tmp/pmc_c.log 2>&1 || { tail -40 /tmp/pmc_c.log > $R/gpurun_out/r4_fused_pmc_c.err; exit 1; }
python3 $R/tools/pmc_summary.py /tmp/pmc_c $R/gpurun_out/r4_fused_pmc_c.md > /dev/null && head -16 $R/gpurun_out/r4_fused_pmc_c.md
cd $R
timeout -k 10 300 python -u tools/wide_decode_probe.py > gpurun_out/final_wide.jsonl 2>&1 || { tail -20 gpurun_out/final_wide.jsonl; exit 1; }
cat gpurun_out/final_wide.jsonl
