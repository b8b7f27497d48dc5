set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/r2_gputest1.log 2>&1 && \
timeout -k 10 300 python bench.py --steps 2 --warmup 1 --verbose > gpurun_out/r2_bench1.log 2>&1
