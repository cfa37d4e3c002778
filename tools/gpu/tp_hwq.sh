set -e
for q in 1 2; do
  timeout -k 10 300 python -u tools/tp_rehearsal.py --world 8 --model llama3-70b --layers 4 --batch 16 --prompt 64 --steps 8 --cmp-tokens 4 --max-batched 1024 --timeout 280 --hw-queues $q --out gpurun_out/hwq$q > gpurun_out/hwq$q.log 2>&1
  python -c "import json; r=json.load(open('gpurun_out/hwq$q/result.json')); print('hwq', $q, r['decode_ms_per_step_shared_gpu'], r['graph_equals_eager'])"
done
