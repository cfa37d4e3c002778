#!/bin/bash
# round-6 end: Mixtral wave breakdown (grouped prefill GEMM per call), Mixtral and 70B-on-one-GPU
# bench lines, the 8B concurrency sweep
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
cd /tmp && export TMPDIR=/tmp
rm -rf /tmp/prof_mix6
timeout -k 10 500 rocprofv3 --kernel-trace --output-format csv -d /tmp/prof_mix6 -- python3 $R/bench.py --model mixtral-8x7b --steps 1 --warmup 1 > $O/r6_prof_mix.log 2>&1 || { tail -20 $O/r6_prof_mix.log; exit 1; }
python3 $R/tools/step_breakdown.py /tmp/prof_mix6 $O/r6_mixtral_step_breakdown.md > /dev/null || exit 1
head -5 $O/r6_mixtral_step_breakdown.md
cd $R
timeout -k 10 400 python bench.py --model mixtral-8x7b --steps 3 --warmup 1 > $O/r6_end_mixtral.json 2> $O/r6_end_mixtral.err || exit 1
cat $O/r6_end_mixtral.json
timeout -k 10 500 python bench.py --model llama3-70b --steps 1 --warmup 1 > $O/r6_end_70b_tp1.json 2> $O/r6_end_70b_tp1.err || exit 1
cat $O/r6_end_70b_tp1.json
rm -f $O/conc_sweep.jsonl
CONC="128 256 512" STEPS=2 bash tools/gpu/conc_sweep.sh || exit 1
cp $O/conc_sweep.jsonl $O/r6_conc_sweep.jsonl
