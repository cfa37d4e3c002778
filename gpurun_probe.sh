set -e
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python tools/bench_gemm.py 64 2>&1 | tail -12
