#!/bin/bash
# Llama-3-70B TP=8 served through the real entry point under torchrun, 8 ranks on ONE MI355X:
# one /v1/chat/completions and one streaming ExecuteToolStream call, graceful shutdown.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 1000 python -u tools/tp_serve_rehearsal.py --world 8 --model llama3-70b --layers ${LAYERS:-80} \
  --timeout 900 --out gpurun_out/tp8_serve > gpurun_out/tp8_serve.log 2>&1
rc=$?
echo "serve rehearsal rc=$rc"
tail -5 gpurun_out/tp8_serve.log
cat gpurun_out/tp8_serve/serve.json 2>/dev/null
exit $rc
