set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gputest_vfrag.log 2>&1 || { tail -30 gpurun_out/gputest_vfrag.log; exit 1; }
tail -2 gpurun_out/gputest_vfrag.log
timeout -k 10 200 python -u tools/attn_layout_lab.py --libs fold,vfrag --ctx 256,384,512,2048 > gpurun_out/attn_vfrag.log 2>&1 || exit 1
cat gpurun_out/attn_vfrag.log
timeout -k 10 300 python -u bench.py --steps 3 > gpurun_out/bench_vfrag.json 2> gpurun_out/bench_vfrag.err || exit 1
cat gpurun_out/bench_vfrag.json
