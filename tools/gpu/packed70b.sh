set -o pipefail
timeout -k 10 400 python -u -m pytest tests/kernels/test_gemm_prefill.py tests/e2e/test_engine_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/t_packed.log 2>&1 || exit 1
timeout -k 10 600 python bench.py --model llama3-70b --steps 1 --warmup 1 > gpurun_out/bench_70b.json 2> gpurun_out/bench_70b.err
