# headline bench: load generator in its own process vs on the server's event loop
set -o pipefail
timeout -k 10 300 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || exit 1
timeout -k 10 300 python bench.py --client inproc > gpurun_out/bench_inproc.json 2> gpurun_out/bench_inproc.err || exit 1
timeout -k 10 300 python bench.py --mode stream > gpurun_out/bench_stream.json 2> gpurun_out/bench_stream.err
