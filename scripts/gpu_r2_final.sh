#!/bin/bash
# Tree GPU tests, headline bench, then the secondary BASELINE configs (one call).
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:-fin}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_tree_engine.py tests/test_forest_share.py tests/test_gpu_kernels.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/${TAG}_test.log 2>&1 && \
timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --verbose > gpurun_out/${TAG}_bench.log 2>&1 && \
bash scripts/gpu_configs.sh
rc=$?
tail -n 1 gpurun_out/${TAG}_test.log; tail -n 1 gpurun_out/${TAG}_bench.log
exit $rc
