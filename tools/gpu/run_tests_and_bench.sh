#!/bin/bash
# GPU-box driver: the GPU test suite, then (only if pytest ended normally) one short bench run.
# Every GPU step has its own time limit; a crash / timeout stops the script.
set -u
mkdir -p gpurun_out
timeout -k 10 ${TEST_LIMIT:-900} python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread \
  ${PYTEST_ARGS:-} > gpurun_out/gputest.log 2>&1
rc=$?
tail -5 gpurun_out/gputest.log
echo "pytest rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
if [ "${BENCH:-1}" = "1" ]; then
  timeout -k 10 ${BENCH_LIMIT:-400} python -u bench.py ${BENCH_ARGS:-} > gpurun_out/bench.json 2> gpurun_out/bench.err
  brc=$?
  cat gpurun_out/bench.json
  echo "bench rc=$brc"
  exit $brc
fi
exit $rc
