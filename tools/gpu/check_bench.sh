# kernel numerics for the touched kernels, prefill-attention micro-bench, then the headline bench
set -o pipefail
timeout -k 10 300 python -u -m pytest tests/kernels/test_gemm_skinny.py tests/kernels/test_attention.py tests/kernels/test_gemm_prefill.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t_check.log 2>&1 || exit 1
timeout -k 10 200 python tools/bench_prefill_attn.py > gpurun_out/prefill_attn.txt 2>&1 || exit 1
timeout -k 10 300 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err
