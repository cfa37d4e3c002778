set -o pipefail
R=$GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/kernels/test_moe.py tests/kernels/test_gemm_prefill.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t_moe.log 2>&1 || exit 1
timeout -k 10 400 python bench.py --model mixtral-8x7b --steps 2 --warmup 1 > gpurun_out/bench_mix.json 2> gpurun_out/bench_mix.err || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/prof_mix -- python3 $R/bench.py --model mixtral-8x7b --steps 1 --warmup 1 > $R/gpurun_out/prof_mix.log 2>&1
