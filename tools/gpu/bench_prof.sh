# headline bench, then the same bench under a kernel trace (per-step analysis)
set -o pipefail
R=$GRAFT_REPO_ROOT
timeout -k 10 300 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_r2d -- python3 $R/bench.py --steps 1 --warmup 1 > $R/gpurun_out/prof_r2d.log 2>&1
