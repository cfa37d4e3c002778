set -o pipefail
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 500 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/prof_mix2 -- python3 $R/bench.py --model mixtral-8x7b --steps 1 --warmup 1 > $R/gpurun_out/prof_mix2.log 2>&1
