# headline bench under a kernel trace (per-kernel step breakdown) + Mixtral bench
set -o pipefail
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_r2c -- python3 $R/bench.py --steps 1 --warmup 1 > $R/gpurun_out/prof_r2c.log 2>&1 || exit 1
cd $R
timeout -k 10 400 python bench.py --model mixtral-8x7b --steps 2 --warmup 1 > gpurun_out/bench_mix.json 2> gpurun_out/bench_mix.err
