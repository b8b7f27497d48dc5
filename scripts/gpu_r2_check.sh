set -o pipefail
cd $GRAFT_REPO_ROOT
TMOG_TREE_GROUPS=1 timeout -k 10 120 python -u scripts/debug/fp_probe.py > gpurun_out/r2_fp_probe1.log 2>&1 && \
TMOG_TREE_GROUPS=2 timeout -k 10 120 python -u scripts/debug/fp_probe.py > gpurun_out/r2_fp_probe2.log 2>&1 && \
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r2_gputest4.log 2>&1 && \
timeout -k 10 300 python bench.py --steps 2 --warmup 1 --verbose > gpurun_out/r2_bench4.log 2>&1
