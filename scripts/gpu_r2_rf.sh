#!/bin/bash
# RF shared-forest path: GPU tests of the tree engine + forest sharing, headline bench, kernel stats.
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:-rf}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_forest_share.py tests/test_tree_engine.py tests/test_gpu_kernels.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/${TAG}_test.log 2>&1 && \
timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --verbose > gpurun_out/${TAG}_bench.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_prof -o ${TAG} -- python3 bench.py --steps 1 --warmup 1 > gpurun_out/${TAG}_prof.log 2>&1
rc=$?
find gpurun_out -name '*trace*.csv' -delete; find gpurun_out -name '*.db' -delete
tail -n 2 gpurun_out/${TAG}_test.log; tail -n 1 gpurun_out/${TAG}_bench.log
exit $rc
