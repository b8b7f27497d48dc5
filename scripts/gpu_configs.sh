#!/bin/bash
# Secondary BASELINE configs on 1 MI355X + a kernel-stats profile of the multiclass-text run.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u bench.py --config multiclass-text --steps ${STEPS:-2} --warmup 1 --verbose > gpurun_out/cfg_mct.log 2>&1 && \
timeout -k 10 400 python -u bench.py --config lr-rf-1m --steps ${STEPS:-2} --warmup 1 --verbose > gpurun_out/cfg_lrrf.log 2>&1 && \
timeout -k 10 600 python -u bench.py --config regression-100m --steps 1 --warmup 1 --verbose > gpurun_out/cfg_reg.log 2>&1 && \
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/cfg_prof -o mct -- python3 bench.py --config multiclass-text --steps 1 --warmup 0 > gpurun_out/cfg_prof.log 2>&1
rc=$?
find gpurun_out -name '*trace*.csv' -delete; find gpurun_out -name '*.db' -delete
tail -2 gpurun_out/cfg_*.log
exit $rc
