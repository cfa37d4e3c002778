#!/bin/bash
# 4-wave prefill GEMM ablations: the same timing with each lab library (wrong results, timing only)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
out=gpurun_out/pg_abl.jsonl
rm -f $out
timeout -k 10 120 python -u tools/pg_probe.py 4 >> $out 2>&1 || { tail -20 $out; exit 1; }
for v in ${ABL:-pg_noglds pg_nords pg_nobar}; do
  POLYKEY_LIB_LIBPK_KERNELS=$PWD/tools/lab/libpk_kernels_$v.so timeout -k 10 120 python -u tools/pg_probe.py 4 >> $out 2>&1 || { tail -20 $out; exit 1; }
done
grep '^{' $out
