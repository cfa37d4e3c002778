set -e
cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -m pytest tests -m gpu -q -x 2>&1 | tail -30
timeout -k 10 900 python bench.py --steps 2 --warmup 1 2>&1 | tail -3
