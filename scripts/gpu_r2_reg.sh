#!/bin/bash
# regression-100m config (BASELINE config 5) + headline bench.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u bench.py --config regression-100m --steps 1 --warmup 1 --verbose > gpurun_out/reg2.log 2>&1 && \
timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --verbose > gpurun_out/reg2_head.log 2>&1
rc=$?
tail -n 1 gpurun_out/reg2.log; tail -n 1 gpurun_out/reg2_head.log
exit $rc
