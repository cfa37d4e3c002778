#!/bin/bash
# end-of-round numbers: headline unary + stream, Mixtral, 70B on one GPU
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --steps 5 > gpurun_out/fb_unary.json 2> gpurun_out/fb_unary.err || exit 1
timeout -k 10 300 python bench.py --steps 5 --mode stream > gpurun_out/fb_stream.json 2> gpurun_out/fb_stream.err || exit 1
timeout -k 10 300 python bench.py --model mixtral-8x7b --steps 2 > gpurun_out/fb_mix.json 2> gpurun_out/fb_mix.err || exit 1
timeout -k 10 400 python bench.py --model llama3-70b --steps 1 > gpurun_out/fb_70b.json 2> gpurun_out/fb_70b.err
