#!/bin/bash
# LR objective kernel: GPU numerics tests, micro-benchmark at the headline shape, headline bench.
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:-lin}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_linear_kernels.py tests/test_gpu_kernels.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/${TAG}_test.log 2>&1 && \
timeout -k 10 200 python -u benchmarks/bench_linear.py --rows 1000000 --cols 329 --problems 24 > gpurun_out/${TAG}_micro.log 2>&1 && \
timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --verbose > gpurun_out/${TAG}_bench.log 2>&1
rc=$?
tail -n 2 gpurun_out/${TAG}_test.log; tail -n 1 gpurun_out/${TAG}_micro.log; tail -n 1 gpurun_out/${TAG}_bench.log
exit $rc
