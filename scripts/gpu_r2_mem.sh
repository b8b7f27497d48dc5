#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/mem_gputest.log 2>&1 && \
timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --verbose > gpurun_out/mem_bench.log 2>&1 && \
timeout -k 10 600 python -u bench.py --config regression-100m --steps 1 --warmup 1 --verbose > gpurun_out/mem_reg.log 2>&1
rc=$?
tail -n 3 gpurun_out/mem_gputest.log; tail -n 1 gpurun_out/mem_bench.log gpurun_out/mem_reg.log
exit $rc
