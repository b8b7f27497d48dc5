#!/bin/bash
# Headline + the secondary BASELINE configs on 1 MI355X (verbose stage timings), one box.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-all}
timeout -k 10 500 python -u bench.py --steps 2 --warmup 1 --verbose > gpurun_out/${T}_head.log 2>&1 && \
timeout -k 10 600 python -u bench.py --config regression-100m --steps 1 --warmup 1 --verbose > gpurun_out/${T}_reg.log 2>&1 && \
timeout -k 10 400 python -u bench.py --config multiclass-text --steps 2 --warmup 1 --verbose > gpurun_out/${T}_mct.log 2>&1 && \
timeout -k 10 400 python -u bench.py --config lr-rf-1m --steps 2 --warmup 1 --verbose > gpurun_out/${T}_lrrf.log 2>&1
rc=$?
tail -n 2 gpurun_out/${T}_*.log
exit $rc
